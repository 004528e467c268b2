"""pip install -e . : builds the native runtime, launcher and HIP kernels in-tree
(make) and installs the console scripts (parity: setup_tensorflow.py /
setup_pytorch.py of the reference, which drive CMake / torch cpp_extension)."""
import os
import subprocess

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class MakeBuild(build_py):
    def run(self):
        targets = ["all"] if os.environ.get("KUNGFU_BUILD_HIP", "1") == "1" else ["runtime", "launcher"]
        subprocess.check_call(["make", "-C", ROOT, "-j%d" % min(16, os.cpu_count() or 8)] + targets)
        super().run()


setup(
    name="kungfu_amd",
    version="0.1.0",
    description="Adaptive data-parallel training engine for AMD MI355X (KungFu capabilities, ROCm-native)",
    packages=find_packages(include=["kungfu_amd", "kungfu_amd.*"]),
    package_data={"kungfu_amd": ["*.so", "lib/*.so", "tuning/miopen/*"]},
    cmdclass={"build_py": MakeBuild},
    entry_points={"console_scripts": [
        "kungfu-run=kungfu_amd.cmd:run",
        "kungfu-config-server=kungfu_amd.cmd:config_server",
        "kungfu-rrun=kungfu_amd.cmd:rrun",
        "kungfu-distribute=kungfu_amd.cmd:distribute",
    ]},
    python_requires=">=3.8",
)
