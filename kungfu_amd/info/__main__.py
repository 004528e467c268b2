"""python -m kungfu_amd.info -- versions of the pieces kungfu-amd runs on
(parity: python -m kungfu.info, srcs/python/kungfu/info/__main__.py:20-27)."""
import os

import torch

import kungfu_amd
from kungfu_amd._lib import hip_available


def main():
    print("kungfu_amd: %s" % kungfu_amd.__version__)
    print("torch: %s (HIP %s)" % (torch.__version__, torch.version.hip))
    print("GPU available: %s" % torch.cuda.is_available())
    if torch.cuda.is_available():
        print("device: %s x%d" % (torch.cuda.get_device_name(0), torch.cuda.device_count()))
    if hip_available():
        from kungfu_amd._lib import hip

        v = hip().rccl_version()
        print("RCCL: %d.%d.%d" % (v // 10000, (v // 100) % 100, v % 100))
    else:
        print("HIP kernels: not built")
    for k in sorted(os.environ):
        if k.startswith("KUNGFU_") or k.startswith("HIP_") or k.startswith("RCCL_") or k.startswith("NCCL_"):
            print("%s=%s" % (k, os.environ[k]))


if __name__ == "__main__":
    main()
