"""``python -m batchai_retinanet_horovod_coco_amd.bin.mxrun -np N -- python -m ...bin.train ...``"""
import sys

from ..parallel.launcher import main

if __name__ == "__main__":
    sys.exit(main())
