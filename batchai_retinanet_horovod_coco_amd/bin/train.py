#!/usr/bin/env python
"""Training CLI -- the reference's ``train.py`` surface on the MI355X-native stack.

Same subcommands, flags, defaults and argument checks as ``/root/reference/train.py:300-380``
(dataset ``coco|pascal|kitti|oid|csv``; weights group ``--snapshot|--imagenet-weights|--weights|
--no-weights``; ``--backbone``, ``--batch-size``, ``--gpu``, ``--multi-gpu``, ``--multi-gpu-force``,
``--epochs``, ``--steps``, ``--snapshot-path``, ``--tensorboard-dir``, ``--no-snapshots``,
``--no-evaluation``, ``--freeze-backbone``, ``--random-transform``, ``--image-min-side``,
``--image-max-side``), plus a ``synthetic`` dataset and MI355X options (``--dtype``, ``--clip-mode``,
``--bucket-mb``, ``--allreduce-dtype``, ``--workers``, ``--shard-data``, ``--checkpoint-format``,
``--lr``, ``--clipnorm``, ``--seed``, ``--log-every``, ``--no-metric-average``, ``--log-all-ranks``,
``--metrics-jsonl``, ``--stop-on-nan``).

Orchestration follows ``main()`` (``train.py:383-450``): init the data-parallel runtime
(``hvd.init()``), backbone object, generators, model (snapshot or weights), summary, callbacks
(Broadcast -> [MetricAverage] -> rank-0 checkpoint -> rank-0 TensorBoard -> evaluation ->
ReduceLROnPlateau), ``fit_generator``.  Launch N ranks with ``mxrun -np N`` / ``torchrun``.
"""
from __future__ import annotations

import argparse
import json
import functools
import os
import sys
import warnings

if __name__ == "__main__" and __package__ is None:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    __package__ = "batchai_retinanet_horovod_coco_amd.bin"


def makedirs(path):
    os.makedirs(path, exist_ok=True)


# ------------------------------------------------------------------------------------- args
def check_args(parsed_args):
    """Inherent contradictions (reference ``check_args``, train.py:300-326, verbatim rules)."""
    if parsed_args.multi_gpu > 1 and parsed_args.batch_size < parsed_args.multi_gpu:
        raise ValueError(
            "Batch size ({}) must be equal to or higher than the number of GPUs ({})".format(parsed_args.batch_size,
                                                                                             parsed_args.multi_gpu))
    if parsed_args.multi_gpu > 1 and parsed_args.snapshot:
        raise ValueError(
            "Multi GPU training ({}) and resuming from snapshots ({}) is not supported.".format(parsed_args.multi_gpu,
                                                                                                parsed_args.snapshot))
    if parsed_args.multi_gpu > 1 and not parsed_args.multi_gpu_force:
        raise ValueError("Multi-GPU support is experimental, use at own risk! Run with --multi-gpu-force if you wish "
                         "to continue.")
    if "resnet" not in parsed_args.backbone:
        warnings.warn("Using experimental backbone {}. Only resnet50 has been properly tested.".format(
            parsed_args.backbone))
    return parsed_args


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="Simple training script for training a RetinaNet network.")
    subparsers = parser.add_subparsers(help="Arguments for specific dataset types.", dest="dataset_type")
    subparsers.required = True

    coco_parser = subparsers.add_parser("coco")
    coco_parser.add_argument("coco_path", help="Path to dataset directory (ie. /tmp/COCO).")

    pascal_parser = subparsers.add_parser("pascal")
    pascal_parser.add_argument("pascal_path", help="Path to dataset directory (ie. /tmp/VOCdevkit).")

    kitti_parser = subparsers.add_parser("kitti")
    kitti_parser.add_argument("kitti_path", help="Path to dataset directory (ie. /tmp/kitti).")

    def csv_list(string):
        return string.split(",")

    oid_parser = subparsers.add_parser("oid")
    oid_parser.add_argument("main_dir", help="Path to dataset directory.")
    oid_parser.add_argument("--version", help="The current dataset version is v4.", default="v4")
    oid_parser.add_argument("--labels-filter", help="A list of labels to filter.", type=csv_list, default=None)
    oid_parser.add_argument("--annotation-cache-dir", help="Path to store annotation cache.", default=".")
    oid_parser.add_argument("--fixed-labels", help="Use the exact specified labels.", default=False)

    csv_parser = subparsers.add_parser("csv")
    csv_parser.add_argument("annotations", help="Path to CSV file containing annotations for training.")
    csv_parser.add_argument("classes", help="Path to a CSV file containing class label mapping.")
    csv_parser.add_argument("--val-annotations", help="Path to CSV file containing annotations for validation "
                                                      "(optional).")

    syn_parser = subparsers.add_parser("synthetic", help="Device-free synthetic COCO-shaped data (benchmarks/tests).")
    syn_parser.add_argument("--num-images", type=int, default=16)
    syn_parser.add_argument("--height", type=int, default=800)
    syn_parser.add_argument("--width", type=int, default=1333)
    syn_parser.add_argument("--num-classes", type=int, default=80)
    syn_parser.add_argument("--max-boxes", type=int, default=20)

    group = parser.add_mutually_exclusive_group()
    group.add_argument("--snapshot", help="Resume training from a snapshot.")
    group.add_argument("--imagenet-weights", help="Initialize the model with pretrained imagenet weights. This is the "
                                                  "default behaviour.", action="store_const", const=True, default=True)
    group.add_argument("--weights", help="Initialize the model with weights from a file.")
    group.add_argument("--no-weights", help="Don't initialize the model with any weights.", dest="imagenet_weights",
                       action="store_const", const=False)

    parser.add_argument("--calibrate-bn", help="With --no-weights: set the frozen BN statistics from the first "
                                               "training batch (models/calibrate.py), a stand-in for ImageNet "
                                               "statistics.", action="store_true")
    parser.add_argument("--backbone", help="Backbone model used by retinanet.", default="resnet50", type=str)
    parser.add_argument("--batch-size", help="Size of the batches.", default=1, type=int)
    parser.add_argument("--gpu", help="Id of the GPU to use (as reported by rocm-smi).")
    parser.add_argument("--multi-gpu", help="Number of GPUs to use for parallel processing.", type=int, default=0)
    parser.add_argument("--multi-gpu-force", help="Extra flag needed to enable (experimental) multi-gpu support.",
                        action="store_true")
    parser.add_argument("--epochs", help="Number of epochs to train.", type=int, default=50)
    parser.add_argument("--steps", help="Number of steps per epoch.", type=int, default=10000)
    parser.add_argument("--snapshot-path", help="Path to store snapshots of models during training (defaults to "
                                                "'./snapshots')", default="./snapshots")
    parser.add_argument("--tensorboard-dir", help="Log directory for Tensorboard output", default="./logs")
    parser.add_argument("--no-snapshots", help="Disable saving snapshots.", dest="snapshots", action="store_false")
    parser.add_argument("--no-evaluation", help="Disable per epoch evaluation.", dest="evaluation",
                        action="store_false")
    parser.add_argument("--freeze-backbone", help="Freeze training of backbone layers.", action="store_true")
    parser.add_argument("--random-transform", help="Randomly transform image and annotations.", action="store_true")
    parser.add_argument("--image-min-side", help="Rescale the image so the smallest side is min_side.", type=int,
                        default=800)
    parser.add_argument("--image-max-side", help="Rescale the image if the largest side is larger than max_side.",
                        type=int, default=1333)

    # ---- MI355X-native additions
    parser.add_argument("--dtype", choices=["auto", "fp32", "bf16", "fp8"], default="auto",
                        help="Compute dtype (auto: bf16 on GPU, fp32 on CPU; fp8: e4m3 forward convs on the "
                             "scaled fp8 MFMA with bf16 gradients).")
    parser.add_argument("--clip-mode", choices=["local", "global"], default="local",
                        help="local = reference clipnorm-before-allreduce; global = clip the averaged gradient "
                             "(lets the all-reduce overlap the backward pass).")
    parser.add_argument("--bucket-mb", type=float, default=None, help="All-reduce bucket size (HOROVOD_FUSION_THRESHOLD)")
    parser.add_argument("--no-overlap", action="store_true",
                        help="Launch every all-reduce bucket after the backward pass instead of as buckets fill.")
    parser.add_argument("--bench", nargs=2, type=int, metavar=("WARMUP", "STEPS"), default=None,
                        help="Benchmark mode: WARMUP untimed then STEPS timed training steps on the chosen dataset; "
                             "prints one JSON line (images/sec for the whole job) instead of training epochs.")
    parser.add_argument("--allreduce-dtype", choices=["fp32", "bf16", "fp16"], default="fp32")
    parser.add_argument("--lr", type=float, default=1e-5)
    parser.add_argument("--clipnorm", type=float, default=0.001)
    parser.add_argument("--workers", type=int, default=1, help="Data loading workers (Keras default 1).")
    parser.add_argument("--loader", choices=["auto", "thread", "process"], default="auto",
                        help="Worker kind: 'process' decodes in worker processes into a pinned shared-memory arena "
                             "(needs --device-preprocess); 'auto' = process when --device-preprocess, else threads.")
    parser.add_argument("--max-queue-size", type=int, default=10)
    parser.add_argument("--shard-data", action="store_true", help="Rank-strided data sharding (reference: none).")
    parser.add_argument("--checkpoint-format", choices=["h5", "safetensors"], default="h5")
    parser.add_argument("--seed", type=int, default=None)
    parser.add_argument("--log-every", type=int, default=1)
    parser.add_argument("--log-all-ranks", action="store_true", help="Progress bar on every rank (reference).")
    parser.add_argument("--no-metric-average", dest="metric_average", action="store_false",
                        help="Do not average epoch logs over ranks (reference behaviour).")
    parser.add_argument("--metrics-jsonl", default=None, help="Per-step JSONL metrics file.")
    parser.add_argument("--stop-on-nan", action="store_true")
    parser.add_argument("--device", default=None, help="Force a device (cpu / cuda).")
    parser.add_argument("--device-preprocess", action="store_true",
                        help="Normalise/warp/resize/pad training images on the GPU (HIP kernels).")
    parser.add_argument("--pad-multiple", type=int, default=None,
                        help="Pad each batch's H and W up to a multiple of this (shape classes for the conv tuner; "
                             "the extra anchors lie outside every image and are ignored).  Default: 32 (the C5 "
                             "stride) on a GPU, 0 (batch max only, the reference) on the CPU; 128 = the P7 stride.")
    return parser


def parse_args(args):
    return check_args(build_parser().parse_args(args))


# ------------------------------------------------------------------------------ generators
def create_generators(args, shard=None):
    from ..data.transform import random_transform_generator
    if args.random_transform:
        transform_generator = random_transform_generator(
            min_rotation=-0.1, max_rotation=0.1, min_translation=(-0.1, -0.1), max_translation=(0.1, 0.1),
            min_shear=-0.1, max_shear=0.1, min_scaling=(0.9, 0.9), max_scaling=(1.1, 1.1),
            flip_x_chance=0.5, flip_y_chance=0.5)
    else:
        transform_generator = random_transform_generator(flip_x_chance=0.5)
    common = dict(batch_size=args.batch_size, image_min_side=args.image_min_side, image_max_side=args.image_max_side,
                  pad_multiple=getattr(args, "pad_multiple", None) or 0)
    train_kw = dict(common, transform_generator=transform_generator, seed=args.seed, shard=shard)
    validation_generator = None
    if args.dataset_type == "coco":
        from ..data.coco import CocoGenerator
        train_generator = CocoGenerator(args.coco_path, "train2017", **train_kw)
        if args.evaluation:
            validation_generator = CocoGenerator(args.coco_path, "val2017", **common)
    elif args.dataset_type == "pascal":
        from ..data.pascal_voc import PascalVocGenerator
        train_generator = PascalVocGenerator(args.pascal_path, "trainval", **train_kw)
        if args.evaluation:
            validation_generator = PascalVocGenerator(args.pascal_path, "test", **common)
    elif args.dataset_type == "csv":
        from ..data.csv_generator import CSVGenerator
        train_generator = CSVGenerator(args.annotations, args.classes, **train_kw)
        if args.val_annotations:
            validation_generator = CSVGenerator(args.val_annotations, args.classes, **common)
    elif args.dataset_type == "oid":
        from ..data.open_images import OpenImagesGenerator
        oid = dict(version=args.version, labels_filter=args.labels_filter,
                   annotation_cache_dir=args.annotation_cache_dir, fixed_labels=args.fixed_labels)
        train_generator = OpenImagesGenerator(args.main_dir, subset="train", **oid, **train_kw)
        if args.evaluation:
            validation_generator = OpenImagesGenerator(args.main_dir, subset="validation", **oid, **common)
    elif args.dataset_type == "kitti":
        from ..data.kitti import KittiGenerator
        train_generator = KittiGenerator(args.kitti_path, subset="train", **train_kw)
        if args.evaluation:
            validation_generator = KittiGenerator(args.kitti_path, subset="val", **common)
    elif args.dataset_type == "synthetic":
        from ..data.synthetic import SyntheticGenerator
        syn = dict(num_images=args.num_images, height=args.height, width=args.width, num_classes=args.num_classes,
                   max_boxes=args.max_boxes)
        train_generator = SyntheticGenerator(data_seed=args.seed or 0, **syn, **train_kw)
        if args.evaluation:
            validation_generator = SyntheticGenerator(data_seed=(args.seed or 0) + 1, **syn, **common)
    else:
        raise ValueError("Invalid data type received: {}".format(args.dataset_type))
    return train_generator, validation_generator


# -------------------------------------------------------------------------------- callbacks
def create_callbacks(trainer, prediction_model, validation_generator, args):
    from ..parallel import callbacks as hvd_callbacks
    from ..parallel import runtime
    from ..train import callbacks as kc
    from ..eval.callbacks import CocoEval, Evaluate
    rank = runtime.rank()
    callbacks = [hvd_callbacks.BroadcastGlobalVariablesCallback(0)]
    if args.metric_average and runtime.size() > 1:
        callbacks.append(hvd_callbacks.MetricAverageCallback())
    if rank == 0 and args.snapshots:
        makedirs(args.snapshot_path)
        ext = "safetensors" if args.checkpoint_format == "safetensors" else "h5"
        callbacks.append(kc.ModelCheckpoint(os.path.join(args.snapshot_path, "checkpoint-{epoch:02d}." + ext)))
    tensorboard_callback = None
    if args.tensorboard_dir and rank == 0:
        tensorboard_callback = kc.TensorBoard(log_dir=args.tensorboard_dir, histogram_freq=0,
                                              batch_size=args.batch_size, write_graph=True)
        callbacks.append(tensorboard_callback)
    if args.evaluation and validation_generator:
        if args.dataset_type == "coco":
            evaluation = CocoEval(validation_generator, tensorboard=tensorboard_callback)
        else:
            evaluation = Evaluate(validation_generator, tensorboard=tensorboard_callback)
        callbacks.append(kc.RedirectModel(evaluation, prediction_model))
    if args.metrics_jsonl and rank == 0:
        callbacks.append(kc.JSONLMetrics(args.metrics_jsonl, every=args.log_every, batch_size=args.batch_size,
                                         world=runtime.size()))
    if args.stop_on_nan:
        callbacks.append(kc.TerminateOnNaN())
    callbacks.append(kc.ReduceLROnPlateau(monitor="loss", factor=0.1, patience=2, verbose=1, mode="auto",
                                          epsilon=0.0001, cooldown=0, min_lr=0))
    return callbacks


def model_summary(model) -> str:
    from ..io.checkpoint import keras_layers
    lines = ["Layer (name)                                 Params", "=" * 58]
    total = trainable = 0
    for name, ws in keras_layers(model).items():
        n = sum(t.numel() for _, t, _ in ws)
        tr = sum(t.numel() for _, t, _ in ws if isinstance(t, __import__("torch").nn.Parameter) and t.requires_grad)
        total += n
        trainable += tr
        lines.append("{:<44} {:>12,}".format(name, n))
    lines += ["=" * 58, "Total params: {:,}".format(total), "Trainable params: {:,}".format(trainable),
              "Non-trainable params: {:,}".format(total - trainable)]
    return "\n".join(lines)


def tower_batch(total: int, towers: int, rank: int) -> int:
    """Images of tower ``rank`` when ``--multi-gpu towers`` splits a ``total``-image batch: ``total // towers`` each,
    the remainder to the lowest ranks -- the global batch stays ``--batch-size``, as Keras ``multi_gpu_model`` slices
    every batch over its towers (/root/reference/train.py:86-89; check_args guarantees ``total >= towers``)."""
    return total // towers + (1 if rank < total % towers else 0)


def _spawn_multi_gpu(args_list, n: int, batch_size: int) -> int:
    """``--multi-gpu N`` = N local ranks of the same data-parallel engine, each training on its
    tower's slice of ``--batch-size`` (``MXR_TOWERS`` = "N:B", read back in main()).  One difference from the
    reference's single-graph towers: the focal loss normaliser (the positive-anchor count) is per tower, then the
    gradients are averaged, where ``multi_gpu_model`` concatenated the tower outputs and normalised over the whole
    batch."""
    from ..parallel.launcher import launch
    argv = []
    skip = False
    for a in args_list:
        if skip:
            skip = False
            continue
        if a == "--multi-gpu":
            skip = True
            continue
        if a.startswith("--multi-gpu=") or a == "--multi-gpu-force":
            continue
        argv.append(a)
    env = dict(os.environ, MXR_TOWERS="%d:%d" % (n, batch_size))
    return launch(n, [sys.executable, "-m", "batchai_retinanet_horovod_coco_amd.bin.train"] + argv, env=env)


# ------------------------------------------------------------------------------------- main
def main(args=None):
    if args is None:
        args = sys.argv[1:]
    raw = list(args)
    args = parse_args(args)

    from ..parallel import runtime
    if args.multi_gpu > 1 and not os.environ.get("MXR_CHILD") and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        return _spawn_multi_gpu(raw, args.multi_gpu, args.batch_size)

    # optionally choose a specific GPU (must happen before the runtime touches HIP)
    if args.gpu:
        if int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", "1"))) > 1:
            warnings.warn("--gpu is ignored with more than one rank (each rank uses its local_rank GPU)")
        else:
            os.environ["HIP_VISIBLE_DEVICES"] = args.gpu
            os.environ["CUDA_VISIBLE_DEVICES"] = args.gpu
    if args.device_preprocess and args.loader != "thread":
        # loader worker processes fork from a server started before anything touches the GPU
        from ..data import process_loader
        process_loader.prestart()
    runtime.init(device=args.device)

    import torch
    from .. import models
    from ..io import checkpoint
    from ..parallel.collectives import Compression
    from ..train.engine import Trainer
    from ..train.loop import fit_generator
    from ..utils.runtime_check import check_runtime

    check_runtime()
    if args.seed is not None:
        torch.manual_seed(args.seed)
    backbone = models.backbone(args.backbone)
    rank, world = runtime.rank(), runtime.size()
    towers = os.environ.get("MXR_TOWERS")
    if towers and os.environ.get("MXR_CHILD"):
        n, total = (int(v) for v in towers.split(":"))
        if n != world:
            raise SystemExit("MXR_TOWERS={} but the world has {} rank(s)".format(towers, world))
        args.batch_size = tower_batch(total, n, rank)
    if args.pad_multiple is None:
        args.pad_multiple = 32 if runtime.device().type == "cuda" else 0
    shard = (rank, world) if args.shard_data else None
    train_generator, validation_generator = create_generators(args, shard=shard)

    initial_epoch = 0
    if args.snapshot is not None:
        print("Loading model, this may take a second...")
        model = models.load_model(args.snapshot, backbone_name=args.backbone)
    else:
        weights = args.weights
        if weights is None and args.imagenet_weights:
            weights = backbone.download_imagenet()
        print("Creating model, this may take a second...")
        model = backbone.retinanet(train_generator.num_classes(),
                                   modifier=models.freeze if args.freeze_backbone else None)
        if weights is not None:
            checkpoint.load_weights(model, weights, by_name=True, skip_mismatch=True)
        elif args.calibrate_bn:
            from ..models.calibrate import calibrate_frozen_bn
            batch = train_generator.compute_input_output(train_generator.groups[0])
            n = calibrate_frozen_bn(model, torch.as_tensor(batch["images"]).cpu())
            if rank == 0:
                print("calibrated {} frozen BN layers on the first training batch".format(n))
    if rank == 0 or args.log_all_ranks:
        print(model_summary(model))

    dev = runtime.device()
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.bfloat16}.get(args.dtype) or \
        (torch.bfloat16 if dev.type == "cuda" else torch.float32)
    if args.dtype == "fp8":
        if dev.type != "cuda":
            raise SystemExit("--dtype fp8 needs an MI355X (gfx950 fp8 MFMA)")
        from ..ops import fp8 as _fp8
        _fp8.set_enabled(True)
    comp = {"fp32": Compression.none, "bf16": Compression.bf16, "fp16": Compression.fp16}[args.allreduce_dtype]
    trainer = Trainer(model, lr=args.lr, clipnorm=args.clipnorm, compute_dtype=dtype, clip_mode=args.clip_mode,
                      compression=comp, bucket_bytes=int(args.bucket_mb * 2 ** 20) if args.bucket_mb else None,
                      device=dev, overlap=not args.no_overlap)
    if args.snapshot is not None:
        checkpoint.load_optimizer_h5(model, trainer.base_optimizer, args.snapshot) \
            if not args.snapshot.endswith(".safetensors") else \
            checkpoint.load_safetensors(model, args.snapshot, trainer.base_optimizer)
        initial_epoch = checkpoint.checkpoint_epoch(args.snapshot) or 0
        trainer.on_weights_changed()

    if args.device_preprocess and dev.type == "cuda":
        train_generator.enable_device_preprocess(dev)

    if "vgg" in args.backbone or "densenet" in args.backbone or "mobilenet" in args.backbone:
        from ..ops.anchors import make_shapes_callback
        trainer.shapes_callback = make_shapes_callback(model)

    if args.bench is not None:
        res = _bench(trainer, train_generator, args.bench[0], args.bench[1], dev, world=runtime.size(),
                     workers=args.workers, loader=args.loader, pad_multiple=args.pad_multiple)
        if rank == 0:
            print(json.dumps(res), flush=True)
        runtime.shutdown()
        return 0

    prediction_model = models.retinanet_bbox(model=model)
    prediction_model.compute_dtype = dtype
    callbacks = create_callbacks(trainer, prediction_model, validation_generator, args)
    verbose = 1 if (rank == 0 or args.log_all_ranks) else 0
    history = fit_generator(trainer, train_generator, steps_per_epoch=args.steps, epochs=args.epochs,
                            verbose=verbose, callbacks=callbacks, initial_epoch=initial_epoch,
                            workers=args.workers, max_queue_size=args.max_queue_size, log_every=args.log_every,
                            loader=args.loader)
    runtime.shutdown()
    return history


def _bench(trainer, generator, warmup: int, steps: int, dev, world: int, workers: int = 1, loader: str = "auto",
           pad_multiple: int = 0) -> dict:
    """--bench: time STEPS training steps on batches of the configured generator (host pipeline
    included, as in training), max over ranks."""
    import time
    import torch
    from ..parallel import runtime as _rt
    from ..data.enqueuer import make_enqueuer
    enq = make_enqueuer(generator, workers=max(1, workers), max_queue_size=10, device=trainer.device,
                        loader=loader).start()
    dump = os.environ.get("MXR_STACK_DUMP")     # diagnostics: every thread's stack every N s to stderr
    if dump:
        import faulthandler
        faulthandler.dump_traceback_later(float(dump), repeat=True)
    images = [0]
    wait = [0.0]       # host time blocked on the loader (the data-bound part of the step)

    shapes = set()
    new_shape = [False]
    cur_hw = [None]

    def one():
        tw = time.perf_counter()
        b = enq.get()
        wait[0] += time.perf_counter() - tw
        images[0] += int(b["images"].shape[0])
        hw = tuple(b["images"].shape[1:3])
        new_shape[0] = hw not in shapes
        shapes.add(hw)
        cur_hw[0] = hw
        return trainer.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    try:
        for _ in range(max(1, warmup)):
            one()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        _rt.barrier()
        images[0] = 0
        wait[0] = 0.0
        # steps that met a new batch shape tune its conv keys inside the timed region (the real-JPEG fixture has
        # two orientations; the first sight of the second one can land after the warm-up): per-step GPU time
        # from events, and the steady rate over the steps that tuned nothing
        from ..ops.conv_tuner import TUNER
        marks = []
        t0 = time.perf_counter()
        b0 = len(TUNER.borrowed)
        for _ in range(steps):
            n0 = len(TUNER.timings)         # raced keys (a borrowed shape-class choice is no race)
            e0 = torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else None
            if e0 is not None:
                e0.record()
            i0 = images[0]
            logs = one()
            if e0 is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                marks.append((e0, e1, images[0] - i0, len(TUNER.timings) != n0, new_shape[0], cur_hw[0]))
        if dev.type == "cuda":
            torch.cuda.synchronize()
        _rt.barrier()
        t1 = time.perf_counter()        # the loader's shutdown is not part of the timed steps
    finally:
        enq.stop()
    images = images[0]
    per_rank = images / max(steps, 1)
    gb = torch.tensor([per_rank], dtype=torch.float64, device=dev)
    if _rt.distributed():
        import torch.distributed as dist
        dist.all_reduce(gb)
    global_batch = float(gb.item())
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if _rt.distributed():
        import torch.distributed as dist
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    steady = tuned = step_ms = None
    if marks:
        # per step: the SLOWEST rank's GPU time, and "tuned" if ANY rank tuned in it (MAX over ranks, as for
        # `el`): a whole-job steady rate no rank's own clock can beat
        per = torch.tensor([[a.elapsed_time(b), 1.0 if t else 0.0] for a, b, _, t, _, _ in marks], dtype=torch.float64,
                           device=dev)
        if _rt.distributed():
            import torch.distributed as dist
            dist.all_reduce(per, op=dist.ReduceOp.MAX)
        per = per.cpu().tolist()
        ok = [(ms, m[2]) for (ms, tf), m in zip(per, marks) if tf == 0.0]
        tuned = sum(1 for _, tf in per if tf != 0.0)
        if ok:
            steady = round(sum(n for _, n in ok) * (global_batch / max(per_rank, 1e-9)) /
                           (sum(t for t, _ in ok) * 1e-3), 3)
        ms = sorted(t for t, _ in per)
        step_ms = {"p50": round(ms[len(ms) // 2], 3), "p90": round(ms[int(0.9 * (len(ms) - 1))], 3),
                   "max": round(ms[-1], 3),
                   "new_shape_steps": [round(t, 1) for (t, tf), m in zip(per, marks) if m[4] and tf == 0.0]}
        if os.environ.get("MXR_BENCH_STEPS_DETAIL") == "1":
            by = {}
            for (t, tf), m in zip(per, marks):
                by.setdefault("%dx%d" % m[5], []).append(round(t, 1))
            step_ms["by_shape"] = by
    return {"metric": "train images/sec (whole job)", "value": round(global_batch * steps / el, 3), "steps": steps,
            "per_rank_batch": per_rank, "global_batch": global_batch,
            "steady_value": steady, "tuned_steps": tuned, "step_ms": step_ms, "borrowed_keys": len(TUNER.borrowed) - b0,
            "raced_keys": len(TUNER.timings), "batch_shapes": len(shapes), "pad_multiple": pad_multiple,
            "warmup": warmup, "ms_per_step": round(1000 * el / max(steps, 1), 3), "n_ranks": world,
            "loss": float(logs["loss"]), "loader": type(enq).__name__, "workers": workers,
            "loader_wait_ms": round(1000 * wait[0] / max(steps, 1), 3),
            "loader_wait_frac": round(wait[0] / max(t1 - t0, 1e-9), 4)}


if __name__ == "__main__":
    r = main()
    sys.exit(r if isinstance(r, int) else 0)
