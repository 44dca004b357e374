#!/usr/bin/env python
"""Run bench.py with module-level switches flipped (same-process A/B of a feature that has no environment knob):

    bench_switch.py ops.conv_launch.FOCAL_FUSED=0 ops.fp8.F8_ONLY_TOWERS=0 -- [bench.py args]"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    sep = argv.index("--") if "--" in argv else len(argv)
    for a in argv[:sep]:
        name, val = a.split("=", 1)
        mod, attr = name.rsplit(".", 1)
        m = importlib.import_module("batchai_retinanet_horovod_coco_amd." + mod)
        if not hasattr(m, attr):
            raise SystemExit("no switch %s" % name)
        setattr(m, attr, type(getattr(m, attr))(int(val)) if isinstance(getattr(m, attr), bool) else val)
    sys.argv = ["bench.py"] + argv[sep + 1:]
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
