"""Checkpoints in the reference's Keras HDF5 layout (plus a fast safetensors format).

Reference behaviour (``/root/reference/train.py:75-78,112-114,404-408``):

* rank 0 writes ``<snapshot_path>/checkpoint-{epoch:02d}.h5`` every epoch (1-based epoch);
* file = ``model.save``: root attrs ``keras_version``, ``backend``, ``model_config``,
  ``training_config``; group ``model_weights`` (attr ``layer_names``; one group per layer with
  attr ``weight_names`` and datasets ``<layer>/<weight>:0``, conv kernels HWIO, BN
  gamma/beta/moving_mean/moving_variance, nested submodels); group ``optimizer_weights``
  (Adam ``iterations``, m, v, vhat placeholders);
* ``--weights`` = ``load_weights(by_name=True, skip_mismatch=True)``; ``--snapshot`` =
  ``models.load_model`` (weights + optimizer).  Unlike the reference, resume also restores the
  epoch (``initial_epoch``) and keeps the DistributedOptimizer.

Internally kernels are OHWI; conversion to/from Keras HWIO happens here.  Writes are atomic
(tmp + rename, in :mod:`.hdf5`).
"""
from __future__ import annotations

import json
import os
import re
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import hdf5

KERAS_VERSION = "2.2.4"
FRAMEWORK = "batchai_retinanet_horovod_coco_amd"


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().float().cpu().numpy()


def keras_layers(model) -> "OrderedDict[str, List[Tuple[str, torch.Tensor, str]]]":
    """Ordered Keras layers with weights: layer -> [(weight_name, tensor, kind)].

    kind: 'kernel' (OHWI <-> HWIO), 'oihw' (torch OIHW <-> HWIO), 'dw' (depthwise (C,1,kh,kw) <->
    (kh,kw,C,1)), 'plain'.
    """
    layers: "OrderedDict[str, list]" = OrderedDict()
    if hasattr(model.backbone, "keras_layers"):
        layers.update(model.backbone.keras_layers())

    def conv(c, prefix=""):
        ws = [(prefix + c.keras_name + "/kernel:0", c.weight, "kernel")]
        if c.bias is not None:
            ws.append((prefix + c.keras_name + "/bias:0", c.bias, "plain"))
        return ws

    def bn(b):
        return [(b.keras_name + "/" + n, t, "plain") for n, t in b.keras_weights()]

    bb = model.backbone
    for c in ([] if hasattr(bb, "keras_layers") else bb.convs()):
        layers[c.keras_name] = conv(c)
        if c.bn is not None:
            layers[c.bn.keras_name] = bn(c.bn)
    for c in model.fpn.convs():
        layers[c.keras_name] = conv(c)
    for sub in (model.regression_submodel, model.classification_submodel):
        ws = []
        for c in sub.convs():
            ws.extend(conv(c))
        layers[sub.keras_name] = ws
    return layers


def model_config(model) -> Dict:
    return {"class_name": "RetinaNet", "framework": FRAMEWORK,
            "config": {"name": "retinanet", "backbone": model.backbone_name, "num_classes": model.num_classes,
                       "num_anchors": model.num_anchors,
                       "layers": list(keras_layers(model).keys())}}


def training_config(optimizer) -> Dict:
    cfg = optimizer.get_config() if optimizer is not None else {}
    return {"optimizer_config": {"class_name": "Adam", "config": cfg},
            "loss": {"regression": "_smooth_l1", "classification": "_focal"},
            "metrics": [], "sample_weight_mode": None, "loss_weights": None}


_TO_KERAS = {"kernel": (1, 2, 3, 0), "oihw": (2, 3, 1, 0), "dw": (2, 3, 0, 1)}
_FROM_KERAS = {"kernel": (3, 0, 1, 2), "oihw": (3, 2, 0, 1), "dw": (2, 3, 0, 1)}


def _to_keras(a: np.ndarray, kind: str) -> np.ndarray:
    return np.transpose(a, _TO_KERAS[kind]) if kind in _TO_KERAS else a


def _from_keras(a: np.ndarray, kind: str) -> np.ndarray:
    if kind in _FROM_KERAS:
        if a.ndim != 4:
            raise ValueError("kernel has rank {}".format(a.ndim))
        return np.transpose(a, _FROM_KERAS[kind])
    return a


def _keras_order_params(model) -> List[Tuple[torch.Tensor, str]]:
    out = []
    for _, ws in keras_layers(model).items():
        for _, t, kind in ws:
            if isinstance(t, torch.nn.Parameter) and t.requires_grad:
                out.append((t, kind))
    return out


def _flat_slice(flat, p):
    seg = flat.by_param[id(p)]
    return seg.offset, seg.numel


def save_keras_h5(path: str, model, optimizer=None, epoch: Optional[int] = None, include_optimizer: bool = True) -> str:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with hdf5.File(path, "w") as f:
        f.attrs["keras_version"] = KERAS_VERSION.encode()
        f.attrs["backend"] = b"tensorflow"
        f.attrs["model_config"] = json.dumps(model_config(model)).encode()
        if optimizer is not None:
            f.attrs["training_config"] = json.dumps(training_config(optimizer)).encode()
        if epoch is not None:
            f.attrs["epoch"] = np.int64(epoch)
        mw = f.create_group("model_weights")
        layers = keras_layers(model)
        hdf5.save_attributes_to_hdf5_group(mw, "layer_names", [n.encode() for n in layers])
        mw.attrs["backend"] = b"tensorflow"
        mw.attrs["keras_version"] = KERAS_VERSION.encode()
        for lname, ws in layers.items():
            g = mw.create_group(lname)
            hdf5.save_attributes_to_hdf5_group(g, "weight_names", [w[0].encode() for w in ws])
            for wname, t, kind in ws:
                a = _to_keras(_np(t), kind)
                g.create_dataset(wname, data=a.astype(np.float32))
        if include_optimizer and optimizer is not None and hasattr(optimizer, "m"):
            ow = f.create_group("optimizer_weights")
            params = _keras_order_params(model)
            names = ["Adam/iterations:0"]
            ow.create_dataset("Adam/iterations:0", data=np.array(int(optimizer.iterations), dtype=np.int64))
            n = len(params)
            flat = optimizer.flat
            for slot, buf in (("m", optimizer.m), ("v", optimizer.v)):
                for i, (p, kind) in enumerate(params):
                    idx = i if slot == "m" else n + i
                    name = "training/Adam/Variable{}:0".format("" if idx == 0 else "_{}".format(idx))
                    off, num = _flat_slice(flat, p)
                    a = _to_keras(buf[off:off + num].detach().cpu().numpy().reshape(p.shape), kind)
                    ow.create_dataset(name, data=a)
                    names.append(name)
            for i in range(n):
                name = "training/Adam/Variable_{}:0".format(2 * n + i)
                ow.create_dataset(name, data=np.zeros((1,), dtype=np.float32))
                names.append(name)
            hdf5.save_attributes_to_hdf5_group(ow, "weight_names", [x.encode() for x in names])
    return path


def _layer_weights_from_file(f) -> "OrderedDict[str, List[Tuple[str, np.ndarray]]]":
    root = f["model_weights"] if "model_weights" in f else f
    names = hdf5.load_attributes_from_hdf5_group(root, "layer_names")
    out = OrderedDict()
    for ln in names:
        g = root[ln]
        wn = hdf5.load_attributes_from_hdf5_group(g, "weight_names")
        out[ln] = [(w, np.asarray(g[w])) for w in wn]
    return out


def load_weights(model, path: str, by_name: bool = True, skip_mismatch: bool = False) -> List[str]:
    """Keras ``load_weights`` (HDF5 or safetensors).  Returns the list of skipped weights."""
    if path.endswith(".safetensors"):
        return load_safetensors(model, path, optimizer=None, skip_mismatch=skip_mismatch)[1]
    f = hdf5.File(path, "r")
    file_layers = _layer_weights_from_file(f)
    layers = keras_layers(model)
    skipped = []
    if not by_name:
        wl = [l for l in layers if layers[l]]
        fl = [l for l in file_layers if file_layers[l]]
        if len(wl) != len(fl):
            raise ValueError("You are trying to load a weight file containing {} layers into a model with {} layers."
                             .format(len(fl), len(wl)))
        pairs = list(zip(wl, fl))
    else:
        pairs = [(l, l) for l in layers if l in file_layers]
    with torch.no_grad():
        for mine, theirs in pairs:
            ws, fws = layers[mine], file_layers[theirs]
            if len(ws) != len(fws):
                msg = "Layer '{}' expects {} weights, but the saved weights have {} elements.".format(mine, len(ws),
                                                                                                  len(fws))
                if skip_mismatch:
                    skipped.append(mine)
                    continue
                raise ValueError(msg)
            for (wname, t, kind), (fname, arr) in zip(ws, fws):
                a = _from_keras(arr, kind)
                if tuple(a.shape) != tuple(t.shape):
                    if skip_mismatch:
                        skipped.append(wname)
                        continue
                    raise ValueError("Layer '{}' weight shape {} does not match saved shape {}".format(
                        mine, tuple(t.shape), tuple(a.shape)))
                t.data.copy_(torch.from_numpy(np.ascontiguousarray(a)).to(t.device, t.dtype))
    return skipped


def load_optimizer_h5(model, optimizer, path: str) -> bool:
    f = hdf5.File(path, "r")
    if "optimizer_weights" not in f:
        return False
    ow = f["optimizer_weights"]
    names = hdf5.load_attributes_from_hdf5_group(ow, "weight_names")
    params = _keras_order_params(model)
    n = len(params)
    if len(names) < 1 + 2 * n:
        return False
    optimizer.iterations = int(np.asarray(ow[names[0]]).reshape(-1)[0])
    flat = optimizer.flat
    with torch.no_grad():
        for slot, buf in (("m", optimizer.m), ("v", optimizer.v)):
            for i, (p, kind) in enumerate(params):
                idx = 1 + (i if slot == "m" else n + i)
                a = _from_keras(np.asarray(ow[names[idx]]), kind)
                off, num = _flat_slice(flat, p)
                buf[off:off + num].copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(buf.device))
    return True


def read_model_config(path: str) -> Dict:
    if path.endswith(".safetensors"):
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
        return json.loads(meta.get("model_config", "{}"))
    f = hdf5.File(path, "r")
    raw = f.attrs.get("model_config")
    return json.loads(bytes(raw).decode()) if raw is not None else {}


def checkpoint_epoch(path: str) -> Optional[int]:
    """Epoch stored in the checkpoint (attribute), else parsed from ``checkpoint-NN``."""
    try:
        if path.endswith(".safetensors"):
            from safetensors import safe_open
            with safe_open(path, framework="pt") as f:
                meta = f.metadata() or {}
            if "epoch" in meta:
                return int(meta["epoch"])
        else:
            f = hdf5.File(path, "r")
            if "epoch" in f.attrs:
                return int(np.asarray(f.attrs["epoch"]).reshape(-1)[0])
    except Exception:  # noqa: BLE001
        pass
    m = re.search(r"(\d+)\.(h5|safetensors)$", os.path.basename(path))
    return int(m.group(1)) if m else None


def load_model(filepath: str, backbone_name: str = "resnet50", **kwargs):
    """``models.load_model``: rebuild the architecture from the stored config, load weights."""
    from .. import models
    cfg = read_model_config(filepath).get("config", {})
    name = cfg.get("backbone", backbone_name)
    model = models.backbone(name).retinanet(int(cfg.get("num_classes", kwargs.get("num_classes", 80))))
    load_weights(model, filepath, by_name=True, skip_mismatch=False)
    return model


# ------------------------------------------------------------------------------ safetensors
def save_safetensors(path: str, model, optimizer=None, epoch: Optional[int] = None) -> str:
    from safetensors.torch import save_file
    tensors = {k: v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    meta = {"model_config": json.dumps(model_config(model)), "framework": FRAMEWORK}
    if epoch is not None:
        meta["epoch"] = str(int(epoch))
    if optimizer is not None and hasattr(optimizer, "m"):
        tensors["__optimizer__.m"] = optimizer.m.detach().cpu()
        tensors["__optimizer__.v"] = optimizer.v.detach().cpu()
        meta["iterations"] = str(int(optimizer.iterations))
        meta["lr"] = repr(float(optimizer.lr))
        meta["training_config"] = json.dumps(training_config(optimizer))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)
    return path


def load_safetensors(model, path: str, optimizer=None, skip_mismatch: bool = False):
    from safetensors.torch import load_file
    from safetensors import safe_open
    sd = load_file(path)
    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
    own = model.state_dict()
    skipped = []
    with torch.no_grad():
        for k, v in own.items():
            if k not in sd or tuple(sd[k].shape) != tuple(v.shape):
                if skip_mismatch:
                    skipped.append(k)
                    continue
                raise ValueError("missing or mismatched tensor {}".format(k))
            v.copy_(sd[k].to(v.device, v.dtype))
        if optimizer is not None and "__optimizer__.m" in sd and sd["__optimizer__.m"].numel() == optimizer.m.numel():
            optimizer.m.copy_(sd["__optimizer__.m"].to(optimizer.m.device))
            optimizer.v.copy_(sd["__optimizer__.v"].to(optimizer.v.device))
            optimizer.iterations = int(meta.get("iterations", 0))
            if "lr" in meta:
                optimizer.lr = float(meta["lr"])
    return meta, skipped


def save_checkpoint(path: str, model, optimizer=None, epoch: Optional[int] = None, fmt: str = "h5") -> str:
    if fmt == "safetensors" or path.endswith(".safetensors"):
        return save_safetensors(path, model, optimizer, epoch)
    return save_keras_h5(path, model, optimizer, epoch)


def restore_checkpoint(path: str, model, optimizer=None) -> Optional[int]:
    """Weights (+ optimizer state when present).  Returns the stored epoch."""
    if path.endswith(".safetensors"):
        load_safetensors(model, path, optimizer)
    else:
        load_weights(model, path, by_name=True)
        if optimizer is not None:
            load_optimizer_h5(model, optimizer, path)
    return checkpoint_epoch(path)
