"""Quick single-GPU probe of ResNet-50 training-step variants (measurement aid).

Usage: python tools/probe_resnet.py --variants autocast_cl,bf16_cl --batch 256
Prints one JSON line per variant with img/s.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from kungfu_amd.models.resnet import resnet50


def run(variant: str, batch: int, steps: int, warmup: int):
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    cl = "_cl" in variant
    model = resnet50().to(dev)
    if cl:
        model = model.to(memory_format=torch.channels_last)
    pure_bf16 = variant.startswith("bf16")
    if pure_bf16:
        model = model.to(torch.bfloat16)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9,
                          foreach=True)
    x = torch.randn(batch, 3, 224, 224, device=dev)
    if cl:
        x = x.to(memory_format=torch.channels_last)
    if pure_bf16:
        x = x.to(torch.bfloat16)
    y = torch.randint(0, 1000, (batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        if variant.startswith("autocast"):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x)
            loss = F.cross_entropy(out.float(), y)
        else:
            out = model(x)
            loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()

    t0 = time.time()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    tw = time.time() - t0
    t0 = time.time()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.time() - t0
    r = {"variant": variant, "batch": batch, "img_s": batch * steps / dt,
         "ms_step": 1000 * dt / steps, "warmup_s": tw}
    print(json.dumps(r), flush=True)
    return r


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="autocast_cl,bf16_cl,autocast")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--benchmark", type=int, default=1)
    a = p.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    print(json.dumps({"device": torch.cuda.get_device_name(0),
                      "torch": torch.__version__,
                      "miopen_find_mode": os.environ.get("MIOPEN_FIND_MODE")}), flush=True)
    for v in a.variants.split(","):
        run(v, a.batch, a.steps, a.warmup)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
