"""Single-layer perceptron used by the MNIST convergence regression.

Parity: ``tests/python/integration/test_mnist_slp.py:10-65`` -- zero-initialised
weights, bias 0.1, softmax + cross-entropy, plain GD lr 0.1.
"""
import torch
import torch.nn as nn


class SLP(nn.Module):
    def __init__(self, input_size: int = 28 * 28, logits: int = 10):
        super().__init__()
        self.fc = nn.Linear(input_size, logits)
        with torch.no_grad():
            self.fc.weight.zero_()
            self.fc.bias.fill_(0.1)

    def forward(self, x):
        return self.fc(x.reshape(x.shape[0], -1))
