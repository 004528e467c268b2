"""Run bench.py with module attributes overridden (same-box A/B of settled-off paths).

    python tools/bench_switch.py kungfu_amd.ops.fused_block:_INLAUNCH_FIN=True -- --steps 20 --warmup 5

Each ``module:attr=value`` is imported and set before bench.main() runs (value parsed as a Python
literal).  Only for measurements: the switches named here are dev paths, not user knobs.
"""
import ast
import importlib
import os
import sys


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets, rest = argv[:cut], argv[cut + 1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    for s in sets:
        lhs, val = s.split("=", 1)
        mod, attr = lhs.split(":")
        m = importlib.import_module(mod)
        if not hasattr(m, attr):
            raise SystemExit("bench_switch: %s has no attribute %s" % (mod, attr))
        setattr(m, attr, ast.literal_eval(val))
        print("bench_switch: %s.%s = %r" % (mod, attr, getattr(m, attr)), file=sys.stderr, flush=True)
    import bench

    sys.argv = ["bench.py"] + rest
    bench.main()


if __name__ == "__main__":
    main()
