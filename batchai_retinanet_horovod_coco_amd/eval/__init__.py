"""Evaluation: COCO bbox COCOeval re-implementation, VOC-style mAP, evaluation callbacks."""
