"""Evaluation callbacks: ``Evaluate`` (VOC mAP) and ``CocoEval`` (12 COCO stats).

Reference: wrapped in ``RedirectModel(..., prediction_model)`` and appended when
``--evaluation`` and a validation generator exist (``/root/reference/train.py:133-142``).
The reference runs them on EVERY rank; here only rank 0 evaluates (others skip), fixing
reference quirk #6; metrics go to the TensorBoard callback and into the epoch logs.
"""
from __future__ import annotations

from ..parallel import runtime
from ..train.callbacks import Callback
from . import coco_eval, voc_eval


def _is_root() -> bool:
    return not runtime.is_initialized() or runtime.rank() == 0


class Evaluate(Callback):
    def __init__(self, generator, iou_threshold=0.5, score_threshold=0.05, max_detections=100, save_path=None,
                 tensorboard=None, verbose=1):
        super().__init__()
        self.generator = generator
        self.iou_threshold = iou_threshold
        self.score_threshold = score_threshold
        self.max_detections = max_detections
        self.save_path = save_path
        self.tensorboard = tensorboard
        self.verbose = verbose

    def on_epoch_end(self, epoch, logs=None):
        logs = logs if logs is not None else {}
        if not _is_root():
            return
        aps = voc_eval.evaluate(self.generator, self.model, iou_threshold=self.iou_threshold,
                                score_threshold=self.score_threshold, max_detections=self.max_detections,
                                save_path=self.save_path)
        self.mean_ap = voc_eval.mean_average_precision(aps)
        if self.verbose:
            for label, (ap, n) in aps.items():
                print("{:.0f} instances of class".format(n), self.generator.label_to_name(label),
                      "with average precision: {:.4f}".format(ap))
            print("mAP: {:.4f}".format(self.mean_ap))
        if self.tensorboard is not None:
            self.tensorboard.add_scalars({"mAP": self.mean_ap}, epoch)
        logs["mAP"] = self.mean_ap


class CocoEval(Callback):
    def __init__(self, generator, tensorboard=None, threshold=0.05):
        super().__init__()
        self.generator = generator
        self.threshold = threshold
        self.tensorboard = tensorboard

    def on_epoch_end(self, epoch, logs=None):
        logs = logs if logs is not None else {}
        if not _is_root():
            return
        stats = coco_eval.evaluate_coco(self.generator, self.model, self.threshold)
        if stats is None:
            return
        scal = {name: float(v) for name, v in zip(coco_eval.STAT_NAMES, stats)}
        if self.tensorboard is not None:
            self.tensorboard.add_scalars(scal, epoch)
        logs.update(scal)
