"""CPU: the bbox COCOeval (eval/coco_eval.py; reference CocoEval callback, /root/reference/train.py:135-138).

The 12 stats of a deterministic toy GT / detection set (tests/fixtures/coco_toy.py: crowd regions, ``ignore`` flags,
all three area ranges, score ties, an image past maxDets=100, images without GT or without detections) are pinned
to the numbers of the round-5 formulation, a line-by-line pycocotools transcription; the current evaluator is a
re-design (one IoU matrix per image/category, native greedy matching, array accumulate).  Parity with pycocotools
itself stays unpinned: it is not installed here."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "fixtures"))
import coco_toy  # noqa: E402

from batchai_retinanet_horovod_coco_amd.data.coco import CocoIndex  # noqa: E402
from batchai_retinanet_horovod_coco_amd.eval.coco_eval import COCOeval, load_results  # noqa: E402
from batchai_retinanet_horovod_coco_amd.utils import cpu_native  # noqa: E402

PINNED = {
    7: [0.194147514195, 0.305184328884, 0.254487698003, 0.312607260726, 0.256244843234, 0.235372465818,
        0.183351023976, 0.398114385614, 0.398114385614, 0.391666666667, 0.444166666667, 0.329166666667],
    11: [0.319568019287, 0.534709178832, 0.36588300412, 0.453623653574, 0.363504704866, 0.27148261177,
         0.265104166667, 0.553348214286, 0.553348214286, 0.523333333333, 0.552301587302, 0.65],
}


@pytest.mark.parametrize("seed", sorted(PINNED))
def test_twelve_stats_pinned(seed):
    gt, dets = coco_toy.build(seed)
    cg = CocoIndex(dataset=gt)
    ev = COCOeval(cg, load_results(cg, dets))
    ev.evaluate()
    ev.accumulate()
    stats = ev.summarize(verbose=False)
    np.testing.assert_allclose(stats, PINNED[seed], rtol=0, atol=1e-9)


def test_native_match_equals_python_fallback(monkeypatch):
    rng = np.random.default_rng(3)
    thr = np.linspace(.5, .95, 10)
    for _ in range(40):
        D, G = rng.integers(0, 12), rng.integers(0, 8)
        iou = rng.uniform(0, 1, (D, G)) * (rng.uniform(0, 1, (D, G)) < 0.6)
        ig = rng.uniform(0, 1, G) < 0.3
        order = np.argsort(ig, kind="stable").astype(np.int32)
        crowd = (rng.uniform(0, 1, G) < 0.2).astype(np.uint8)
        nat = cpu_native.coco_match(iou, order, ig[order], crowd, thr)
        monkeypatch.setattr(cpu_native, "lib", lambda: None)
        py = cpu_native.coco_match(iou, order, ig[order], crowd, thr)
        monkeypatch.undo()
        assert np.array_equal(nat, py)


def test_crowd_gt_matches_repeatedly_and_regular_first():
    # two detections on one crowd region: both matched (and so ignored); a regular gt wins over an ignored one
    iou = np.array([[0.9, 0.6], [0.8, 0.0]])
    order = np.array([1, 0], dtype=np.int32)            # gt 1 regular, gt 0 crowd (ignored) last
    ig = np.array([0, 1], dtype=np.uint8)
    crowd = np.array([1, 0], dtype=np.uint8)
    m = cpu_native.coco_match(iou, order, ig, crowd, np.array([0.5]))
    assert m.tolist() == [[0, 1]]                       # det 0 -> regular gt (0.6), det 1 -> crowd
    m = cpu_native.coco_match(iou, order, ig, crowd, np.array([0.7]))
    assert m.tolist() == [[1, 1]]                       # regular gt below the threshold: both on the crowd
