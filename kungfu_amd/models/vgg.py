"""VGG-16 (the reference's second headline model)."""
import torch
import torch.nn as nn

CFG16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


class VGG(nn.Module):
    def __init__(self, cfg=CFG16, num_classes: int = 1000, batch_norm: bool = False, fused: bool = False):
        """``fused``: conv+bias+ReLU as one ``ops.conv.Conv2dReLU`` (fused bias/ReLU pass on the
        MFMA path); an ``nn.Identity`` keeps the ReLU's slot so state_dict keys do not move."""
        super().__init__()
        if fused and not batch_norm:
            from ..ops.conv import Conv2dReLU
        layers, c = [], 3
        for v in cfg:
            if v == "M":
                if fused and not batch_norm:
                    from ..ops.pool import MaxPool2x2

                    layers.append(MaxPool2x2())
                    continue
                layers.append(nn.MaxPool2d(2, 2))
            else:
                if fused and not batch_norm:
                    layers += [Conv2dReLU(c, v, 3, padding=1), nn.Identity()]
                    c = v
                    continue
                layers.append(nn.Conv2d(c, v, 3, padding=1))
                if batch_norm:
                    layers.append(nn.BatchNorm2d(v))
                layers.append(nn.ReLU(inplace=True))
                c = v
        if fused and not batch_norm:
            # the whole conv/bias/ReLU/pool stack as one autograd node (bias + ReLU inside the
            # conv and pool kernels, ops/vgg_fused.py); same modules, same state_dict keys
            from ..ops.vgg_fused import FusedVGGFeatures

            self.features = FusedVGGFeatures(*layers)
        else:
            self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


def vgg16(fused_bn: bool = False, **kw):
    """``fused_bn`` (the zoo-wide "use the HIP fusions" flag) selects the fused conv+bias+ReLU."""
    return VGG(CFG16, fused=bool(fused_bn), **kw)
