"""VOC-style per-class average precision (keras-retinanet ``utils.eval.evaluate`` behaviour).

Used by the ``Evaluate`` callback for non-COCO datasets (``/root/reference/train.py:139-141``):
detections from the prediction model (score > 0.05, top ``max_detections`` per image), greedy
matching against ground truth with the "+1" IoU (native ``compute_overlap``), cumulative
TP/FP over score-sorted detections, and the all-point interpolated AP (``_compute_ap``).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from ..utils.cpu_native import compute_overlap


def _compute_ap(recall: np.ndarray, precision: np.ndarray) -> float:
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([0.0], precision, [0.0]))
    for i in range(mpre.size - 1, 0, -1):
        mpre[i - 1] = np.maximum(mpre[i - 1], mpre[i])
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


def _get_detections(generator, prediction_model, score_threshold=0.05, max_detections=100):
    from .coco_eval import predict_image
    all_detections = [[None for _ in range(generator.num_classes())] for _ in range(generator.size())]
    for i in range(generator.size()):
        boxes, scores, labels = predict_image(generator, prediction_model, i)
        indices = np.where(scores > score_threshold)[0]
        sc = scores[indices]
        order = np.argsort(-sc)[:max_detections]
        image_boxes = boxes[indices[order], :]
        image_scores = sc[order]
        image_labels = labels[indices[order]]
        dets = np.concatenate([image_boxes, image_scores[:, None], image_labels[:, None]], axis=1)
        for label in range(generator.num_classes()):
            all_detections[i][label] = dets[dets[:, -1] == label, :-1]
    return all_detections


def _get_annotations(generator):
    all_annotations = [[None for _ in range(generator.num_classes())] for _ in range(generator.size())]
    for i in range(generator.size()):
        ann = np.asarray(generator.load_annotations(i)).reshape(-1, 5)
        for label in range(generator.num_classes()):
            all_annotations[i][label] = ann[ann[:, 4] == label, :4].copy()
    return all_annotations


def evaluate_detections(all_detections, all_annotations, num_classes: int,
                        iou_threshold: float = 0.5) -> Dict[int, Tuple[float, float]]:
    average_precisions = {}
    for label in range(num_classes):
        false_positives = []
        true_positives = []
        scores = []
        num_annotations = 0.0
        for i in range(len(all_annotations)):
            detections = all_detections[i][label]
            annotations = all_annotations[i][label]
            num_annotations += annotations.shape[0]
            detected = []
            for d in detections:
                scores.append(d[4])
                if annotations.shape[0] == 0:
                    false_positives.append(1)
                    true_positives.append(0)
                    continue
                overlaps = compute_overlap(np.expand_dims(d[:4], axis=0), annotations)
                assigned = int(np.argmax(overlaps, axis=1)[0])
                max_overlap = overlaps[0, assigned]
                if max_overlap >= iou_threshold and assigned not in detected:
                    false_positives.append(0)
                    true_positives.append(1)
                    detected.append(assigned)
                else:
                    false_positives.append(1)
                    true_positives.append(0)
        if num_annotations == 0:
            average_precisions[label] = (0.0, 0.0)
            continue
        scores = np.asarray(scores)
        order = np.argsort(-scores, kind="mergesort")
        fp = np.cumsum(np.asarray(false_positives, dtype=np.float64)[order])
        tp = np.cumsum(np.asarray(true_positives, dtype=np.float64)[order])
        recall = tp / num_annotations
        precision = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
        average_precisions[label] = (_compute_ap(recall, precision), num_annotations)
    return average_precisions


def evaluate(generator, prediction_model, iou_threshold: float = 0.5, score_threshold: float = 0.05,
             max_detections: int = 100, save_path=None) -> Dict[int, Tuple[float, float]]:
    dets = _get_detections(generator, prediction_model, score_threshold, max_detections)
    anns = _get_annotations(generator)
    return evaluate_detections(dets, anns, generator.num_classes(), iou_threshold)


def mean_average_precision(aps: Dict[int, Tuple[float, float]]) -> float:
    present = [ap for ap, n in aps.values() if n > 0]
    return float(sum(present) / len(present)) if present else 0.0
