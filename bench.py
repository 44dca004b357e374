#!/usr/bin/env python
"""Headline benchmark: training images/sec for the whole node, RetinaNet-R50-FPN at 800x1333.

BASELINE.json metric "images/sec (whole node) RetinaNet-R50-FPN 800px at 1/2/4/8 MI355X",
config "RetinaNet-R50-FPN bf16, 800x1333, batch 16 on one MI355X" (weak scaling: batch 16
per GPU).  Synthetic COCO-shaped data generated on the device, random-init weights
(``--no-weights``).  Every timed step is a complete training step: GPU anchor-target
assignment, forward, focal + smooth-L1, backward, bucketed RCCL all-reduce, clip and
Keras-Adam update.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With ``--gpus N > 1`` and no launcher environment (``WORLD_SIZE`` / ``OMPI_COMM_WORLD_SIZE``),
this process starts the N ranks itself (``parallel.launcher``: plain child processes, started
before anything here touches the GPU) and exits with their status.  Under a launcher the world
size must equal ``--gpus``.  Rank 0 prints ONE JSON line; per-GPU work is fixed (weak scaling) and
``value`` is the whole-job images/sec.  Multi-rank GPU runs reduce gradients through the native
C++ RCCL bucket engine by default (``--comm``); its per-step GPU timings are reported as
``comm_ms`` (summed all-reduce time) and ``comm_exposed_ms`` (the part after the backward).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRIC = "images/sec (whole node) RetinaNet-R50-FPN 800px at 1/2/4/8 MI355X"


def metric_label(backbone: str, height: int, width: int) -> str:
    """BASELINE.json's metric string for its config (R50-FPN at 800x1333); any other backbone / size names its own
    model and input, so a run of another config never reports the headline label."""
    if backbone == "resnet50" and (height, width) == (800, 1333):
        return METRIC
    model = "RetinaNet-{}-FPN".format(backbone.replace("resnet", "R"))
    return "images/sec (whole node) {} {}x{}".format(model, height, width)


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=16)
    p.add_argument("--height", type=int, default=800)
    p.add_argument("--width", type=int, default=1333)
    p.add_argument("--backbone", default="resnet50")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                   help="fp8: forward convs in e4m3 on the scaled fp8 MFMA (bf16 gradients), BASELINE config 5")
    p.add_argument("--clip-mode", default="global", choices=["global", "local"])
    p.add_argument("--allreduce-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--bucket-mb", type=float, default=25.0)
    p.add_argument("--comm", default=None, choices=["auto", "native", "torch"],
                   help="gradient all-reduce engine (sets MXR_COMM): native C++ RCCL bucket engine (default "
                        "for multi-rank GPU runs) or torch ProcessGroupNCCL")
    p.add_argument("--conv-backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--kernels", default="auto", choices=["auto", "off"],
                   help="'off' disables every HIP kernel (pure PyTorch/MIOpen path, for A/B)")
    p.add_argument("--graph", action="store_true", help="capture the step in a HIP graph")
    p.add_argument("--no-calibrate-bn", dest="calibrate_bn", action="store_false",
                   help="keep identity frozen-BN statistics (default: calibrate them on one synthetic image, "
                        "a stand-in for the ImageNet statistics the reference starts from)")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--rccl-debug-dir", default="gpurun_out",
                   help="world > 1: rank 0 writes RCCL's INIT/GRAPH debug log (topology, rings/channels) here "
                        "(NCCL_DEBUG=INFO, NCCL_DEBUG_FILE); '' disables")
    p.add_argument("--profile", choices=["stats", "pmc"], default=None,
                   help="re-run this benchmark as a child under rocprofv3: 'stats' = kernel trace + per-kernel "
                        "statistics (summarised by family), 'pmc' = MFMA / LDS / wait counters (kernel trace only)")
    p.add_argument("--profile-dir", default="gpurun_out/profile")
    return p.parse_args(argv)


PMC = ["SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES",
       "SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"]


def profile(args, argv) -> int:
    """Run the benchmark (minus --profile) as a CHILD process under rocprofv3 -- started before this
    process touches the GPU, the program itself right after '--' (no exec, no launcher hop)."""
    import subprocess
    here = os.path.abspath(__file__)
    out = os.path.abspath(args.profile_dir)
    os.makedirs(out, exist_ok=True)
    rest, skip = [], False
    for a in (argv if argv is not None else sys.argv[1:]):
        if skip:
            skip = False
            continue
        if a in ("--profile", "--profile-dir"):
            skip = True
            continue
        if a.startswith("--profile"):
            continue
        rest.append(a)
    env = dict(os.environ, TMPDIR="/tmp")
    runs = [["--kernel-trace", "--stats"]] if args.profile == "stats" else \
        [["--kernel-trace", "--pmc"] + grp.split() for grp in PMC]
    rc = 0
    for i, flags in enumerate(runs):
        d = os.path.join(out, "run%d" % i)
        cmd = ["rocprofv3"] + flags + ["-d", d, "-o", "run", "--output-format", "csv", "--",
                                       sys.executable, here] + rest
        rc = subprocess.call(cmd, cwd="/tmp", env=env)
        if rc != 0:
            return rc
    if args.profile == "stats":
        import glob
        stats = glob.glob(os.path.join(out, "run0", "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            steps = args.steps + max(args.warmup, 1)
            subprocess.call([sys.executable, os.path.join(os.path.dirname(here), "scripts", "prof_summary.py"),
                             stats[0], "--steps", str(steps)])
    return rc


def _launcher_world():
    for n in ("OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "WORLD_SIZE"):
        v = os.environ.get(n)
        if v:
            return int(v)
    return None


def rccl_debug_env(args, rank: int, world: int) -> None:
    """Multi-rank runs: rank 0 logs RCCL's topology detection and the rings / channels it built (the xGMI
    evidence of SURVEY §2.5), unless the user set NCCL_DEBUG themselves.  Must run before any RCCL
    communicator exists (ProcessGroupNCCL and the native engine both read it at init)."""
    if world <= 1 or rank != 0 or not args.rccl_debug_dir or "NCCL_DEBUG" in os.environ:
        return
    os.makedirs(args.rccl_debug_dir, exist_ok=True)
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH,ENV")
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(os.path.abspath(args.rccl_debug_dir), "rccl_debug_w%d.%%p.log" % world)


def check_rccl(info, world: int):
    """The native engine's communicator must span exactly ``world`` ranks as RCCL itself reports it
    (``ncclCommCount``); returns an error message, or None.  -1 = the library lacks the query."""
    if info is None:
        return None
    n = info.get("nranks", -1)
    if n != -1 and n != world:
        return "RCCL communicator has {} rank(s), expected {} (--gpus)".format(n, world)
    return None


def spawn(args, argv) -> int:
    """Start ``--gpus`` ranks of this benchmark as child processes (this process never touches the
    GPU) and return the first failing exit code."""
    from batchai_retinanet_horovod_coco_amd.parallel.launcher import launch
    rest = list(argv if argv is not None else sys.argv[1:])
    return launch(args.gpus, [sys.executable, os.path.abspath(__file__)] + rest, tag_output=False, capture=False)


def main(argv=None):
    args = parse(argv)
    if args.profile:
        return profile(args, argv)
    if args.comm:
        os.environ["MXR_COMM"] = args.comm
    env_world = _launcher_world()
    if env_world is None and args.gpus > 1:
        return spawn(args, argv)
    if (env_world or 1) != args.gpus:
        print("bench.py: --gpus {} but the launcher started {} rank(s)".format(args.gpus, env_world or 1),
              file=sys.stderr)
        return 2
    from batchai_retinanet_horovod_coco_amd.parallel import runtime
    from batchai_retinanet_horovod_coco_amd.parallel.collectives import Compression
    from batchai_retinanet_horovod_coco_amd import models
    from batchai_retinanet_horovod_coco_amd.ops import conv as conv_ops, native
    from batchai_retinanet_horovod_coco_amd.train.engine import Trainer
    from batchai_retinanet_horovod_coco_amd.data.synthetic import SyntheticBatches

    # MXR_DIST_BACKEND=gloo --comm torch: a multi-rank rehearsal of the full step with several ranks sharing
    # the visible GPU(s) (RCCL refuses two ranks on one device; gloo stages through the host)
    rehearsal = os.environ.get("MXR_DIST_BACKEND") == "gloo"
    if args.gpus > 1 and torch.cuda.is_available() and torch.cuda.device_count() < args.gpus and not rehearsal:
        print("bench.py: --gpus {} but only {} GPU(s) visible (one rank per GPU)".format(
            args.gpus, torch.cuda.device_count()), file=sys.stderr)
        return 2
    rccl_debug_env(args, int(os.environ.get("OMPI_COMM_WORLD_RANK", os.environ.get("RANK", "0"))), args.gpus)
    runtime.init()
    rank, world = runtime.rank(), runtime.size()
    dev = runtime.device()
    assert world == args.gpus, (world, args.gpus)
    if args.kernels == "off":
        native.disable()
    conv_ops.set_conv_backend(args.conv_backend if args.kernels != "off" else "torch")
    if dev.type == "cuda":
        torch.backends.cudnn.benchmark = False     # the per-shape tuner owns algorithm choice
    torch.manual_seed(1234)
    model = models.backbone(args.backbone).retinanet(80)
    if args.calibrate_bn:
        # stand-in for the reference's ImageNet BN statistics (models/calibrate.py); CPU, untimed
        from batchai_retinanet_horovod_coco_amd.models.calibrate import calibrate_from_synthetic
        calibrate_from_synthetic(model, torch.device("cpu"), batch=1, height=384, width=640)
    dtype = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    if args.dtype == "fp8":
        from batchai_retinanet_horovod_coco_amd.ops import fp8 as _fp8
        _fp8.set_enabled(True)
    trainer = Trainer(model, lr=1e-5, clipnorm=0.001, compute_dtype=dtype, clip_mode=args.clip_mode,
                      compression=Compression.bf16 if args.allreduce_dtype == "bf16" else Compression.none,
                      bucket_bytes=int(args.bucket_mb * 1024 * 1024), device=dev)
    rccl = trainer.optimizer.native.info() if trainer.optimizer.native is not None else None
    err = check_rccl(rccl, world)
    if err:
        print("bench.py: " + err, file=sys.stderr)
        runtime.shutdown()
        return 3
    # reference BroadcastGlobalVariablesCallback(0): identical initial weights on every rank
    from batchai_retinanet_horovod_coco_amd.parallel.collectives import broadcast_parameters
    broadcast_parameters(trainer.state_for_broadcast(), 0)
    data = SyntheticBatches(args.batch_size, args.height, args.width, pool=2, device=dev, seed=100 + rank,
                            dtype=dtype if dev.type == "cuda" else torch.float32)

    trainer.on_weights_changed()      # broadcast rewrote the weights: refresh the bf16 compute copies

    def step():
        b = next(data)
        return trainer.train_on_batch(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    graphed = bool(args.graph and dev.type == "cuda" and (not runtime.distributed() or
                                                          trainer.optimizer.native is not None))
    if graphed:
        # warm up eagerly (tuner decisions), then capture the whole step in one HIP graph
        for i in range(max(1, args.warmup)):
            step()
        b0 = next(data)
        replay = trainer.graph_step(b0["images"], b0["gt"], b0["gt_count"], b0["image_hw"], warmup=1)

        def step():  # noqa: F811
            b = next(data)
            return replay(b["images"], b["gt"], b["gt_count"], b["image_hw"])

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        runtime.barrier()

    logs = None
    t_w = time.time()
    from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
    if args.warmup == 0:
        # the per-shape conv tuner times candidates on first sight: never inside the timed region
        step()
        TUNER.sync(0)
    for i in range(args.warmup):
        logs = step()
        if i == 0:
            TUNER.sync(0)      # every rank runs rank 0's kernel choices from here on
        if args.verbose and rank == 0:
            sync()
            print("warmup", i, {k: float(v) for k, v in logs.items()}, "%.1fs" % (time.time() - t_w),
                  file=sys.stderr, flush=True)
    # the model, tuner tables and kernel caches are built: move them out of the cyclic GC's reach, so a full
    # collection during a step walks only that step's objects (an ~1 ms host pause drained the GPU queue once
    # in a profiled run: profiles/r5_final_overlap_517ips.txt) -- the training loop does the same
    import gc
    gc.collect()
    gc.freeze()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        logs = step()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if runtime.distributed():
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    consistent, diverged = None, []
    if world > 1 or trainer.optimizer.native is not None:
        # after the timed region: the replicas must still hold bit-identical weights and Adam slots
        from batchai_retinanet_horovod_coco_amd.parallel.collectives import replicas_consistent
        dopt = trainer.optimizer
        fault = os.environ.get("MXR_TEST_FAULT_REPLICA")
        if fault is not None:
            # test hook (tests/test_comm_agree.py): break one replica.  Honoured only under pytest, so a stray
            # variable can never corrupt a real benchmark
            if "PYTEST_CURRENT_TEST" not in os.environ:
                print("bench: ignoring MXR_TEST_FAULT_REPLICA outside pytest", file=sys.stderr, flush=True)
            elif fault == str(rank):
                print("bench: MXR_TEST_FAULT_REPLICA: breaking rank %d's replica" % rank, file=sys.stderr, flush=True)
                dopt.flat.data[0] += 1.0
        consistent, diverged = replicas_consistent([dopt.flat.data, dopt.optimizer.m])
    comm = trainer.optimizer.comm_stats()
    loss = float(logs["loss"]) if logs is not None else float("nan")
    images = world * args.batch_size * args.steps
    value = images / elapsed
    res = {
        "metric": metric_label(args.backbone, args.height, args.width),
        "value": round(value, 3),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / max(args.steps, 1), 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (device-generated COCO-shaped images + random boxes), random-init weights",
        "config": {"model": "RetinaNet-{}-FPN".format(args.backbone.replace("resnet", "R")),
                   "global_batch": world * args.batch_size, "per_gpu_batch": args.batch_size,
                   "seq_len": None, "image": [args.height, args.width], "parallelism": "dp{}".format(world),
                   "clip_mode": args.clip_mode, "allreduce_dtype": args.allreduce_dtype,
                   "conv_backend": conv_ops.get_conv_backend(), "hip_kernels": native.available(),
                   "hip_graph": graphed,
                   "comm_engine": ("native" if trainer.optimizer.native is not None else
                                   ("torch" if runtime.distributed() else "none")),
                   "comm_fallback": trainer.optimizer._fallback,
                   "replicas_consistent": consistent,
                   "buckets_mb": [round(b / 2 ** 20, 2) for b in trainer.optimizer.bucket_sizes_bytes()],
                   "rccl_nranks": rccl["nranks"] if rccl else None,
                   "rccl_device": rccl["device"] if rccl else None,
                   "final_loss": loss},
    }
    if world > 1:
        from batchai_retinanet_horovod_coco_amd.parallel import xgmi
        # ring model of this bucket list on the 7-link xGMI mesh (parallel/xgmi.py), next to the measured
        # comm_ms / comm_exposed_ms
        res["config"]["comm_model"] = xgmi.plan(trainer.optimizer.bucket_sizes_bytes(), world)
    if comm is not None:
        # GPU timings of the last timed step (timing events around each bucket's all-reduce)
        res["config"]["comm_ms"] = round(comm["comm_ms"], 3)
        res["config"]["comm_exposed_ms"] = round(comm["exposed_ms"], 3)
    try:
        from batchai_retinanet_horovod_coco_amd.ops.conv_tuner import TUNER
        res["config"]["conv_algos"] = TUNER.summary()
        from batchai_retinanet_horovod_coco_amd.ops import conv_launch as _cl
        # forms adopted over a near-tie race winner (ConvTuner.prefer) and launches of the fused focal final
        res["config"]["preferred_forms"] = dict(TUNER.preferred)
        res["config"]["focal_fused_calls"] = _cl.FOCAL_LAUNCHES[0]
        if os.environ.get("MXR_SAVE_CONV_TABLE") and rank == 0:
            TUNER.save(os.environ["MXR_SAVE_CONV_TABLE"])
    except Exception:  # noqa: BLE001
        pass
    if rank == 0:
        print(json.dumps(res), flush=True)
    runtime.shutdown()
    if consistent is False:
        print("bench.py: replicas diverged: rank(s) {} differ from rank 0 (weights / Adam m)".format(diverged),
              file=sys.stderr)
        return 4
    return 0


if __name__ == "__main__":
    sys.exit(main())
