"""Minimal HDF5 writer/reader (the subset Keras ``model.save`` files use).

The reference checkpoints with ``keras.callbacks.ModelCheckpoint`` -> ``model.save`` -> h5py ->
libhdf5 (``/root/reference/train.py:112-114``).  h5py is not available in
this environment, so this module implements the on-disk format directly (HDF5 File Format
Specification, "version 0" structures, the same ones libhdf5 writes with its default
``libver='earliest'`` as h5py does):

* superblock v0; v1 object headers (8-byte aligned messages, continuation messages on read);
* groups as symbol tables: v1 group B-tree (one leaf node, K = 64 -> up to 128 symbol-table
  nodes) + SNOD symbol-table nodes (leaf K = 64 -> 128 entries each) + a local heap of names;
* datasets: dataspace v1, IEEE float / signed integer / fixed-length string datatypes, fill-value
  message v2, contiguous data layout (v3); compact layout and v1/v2 layouts are accepted on read;
* attributes (message v1 on write; v1-v3 on read): fixed-length strings, arrays of strings, numbers.

``File(path, 'w')`` / ``File(path, 'r')`` expose an h5py-like subset: ``create_group``,
``create_dataset``, ``attrs``, ``__getitem__`` with '/' paths, ``keys()``, ``visit``.
Writes go to ``path + '.tmp'`` and are renamed on close (atomic checkpoints).
"""
from __future__ import annotations

import os
import struct
from collections import OrderedDict
from typing import Any, Dict, List, Optional

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIG = b"\x89HDF\r\n\x1a\n"
LEAF_K = 64          # symbol-table node capacity = 2 * LEAF_K entries
BTREE_K = 64         # group B-tree node capacity = 2 * BTREE_K children


def _pad8(n: int) -> int:
    return (n + 7) & ~7


# =========================================================================================
# in-memory tree
# =========================================================================================
class Attrs(OrderedDict):
    pass


class Dataset:
    def __init__(self, name: str, data: np.ndarray, attrs=None):
        self.name = name
        self._data = np.ascontiguousarray(data)
        self.attrs = Attrs(attrs or {})

    @property
    def shape(self):
        return self._data.shape

    @property
    def dtype(self):
        return self._data.dtype

    def __getitem__(self, item):
        return self._data[item]

    def __array__(self, dtype=None):
        return self._data if dtype is None else self._data.astype(dtype)


class Group:
    def __init__(self, name: str = "/"):
        self.name = name
        self.attrs = Attrs()
        self.children: "OrderedDict[str, Any]" = OrderedDict()

    # h5py-like API ------------------------------------------------------------------
    def _walk(self, path: str, create: bool):
        node = self
        parts = [p for p in path.split("/") if p]
        for i, p in enumerate(parts[:-1]):
            if p not in node.children:
                if not create:
                    raise KeyError(path)
                node.children[p] = Group(node.name.rstrip("/") + "/" + p)
            node = node.children[p]
            if not isinstance(node, Group):
                raise KeyError(path)
        return node, parts[-1] if parts else ""

    def create_group(self, path: str) -> "Group":
        parent, leaf = self._walk(path, True)
        if leaf in parent.children:
            g = parent.children[leaf]
            if not isinstance(g, Group):
                raise ValueError("{} exists and is not a group".format(path))
            return g
        g = Group(parent.name.rstrip("/") + "/" + leaf)
        parent.children[leaf] = g
        return g

    def require_group(self, path: str) -> "Group":
        return self.create_group(path)

    def create_dataset(self, path: str, data=None, shape=None, dtype=None) -> Dataset:
        parent, leaf = self._walk(path, True)
        if data is None:
            data = np.zeros(shape, dtype=dtype or np.float32)
        arr = np.asarray(data)
        if dtype is not None:
            arr = arr.astype(dtype)
        ds = Dataset(parent.name.rstrip("/") + "/" + leaf, arr)
        parent.children[leaf] = ds
        return ds

    def __getitem__(self, path: str):
        parent, leaf = self._walk(path, False)
        if leaf == "":
            return self
        return parent.children[leaf]

    def __contains__(self, path: str) -> bool:
        try:
            self[path]
            return True
        except KeyError:
            return False

    def keys(self):
        return list(self.children.keys())

    def items(self):
        return list(self.children.items())

    def __iter__(self):
        return iter(self.children)

    def __len__(self):
        return len(self.children)

    def visit(self, fn, prefix=""):
        for k, v in self.children.items():
            p = prefix + k
            r = fn(p)
            if r is not None:
                return r
            if isinstance(v, Group):
                r = v.visit(fn, p + "/")
                if r is not None:
                    return r
        return None


# =========================================================================================
# datatypes / dataspaces
# =========================================================================================
def _encode_dtype(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            sign = 31
        elif dt.itemsize == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            sign = 63
        elif dt.itemsize == 2:
            props = struct.pack("<HHBBBBI", 0, 16, 10, 5, 0, 10, 15)
            sign = 15
        else:
            raise TypeError(dt)
        return bytes([0x11, 0x20, sign, 0x00]) + struct.pack("<I", dt.itemsize) + props
    if dt.kind in "iu":
        flags = 0x08 if dt.kind == "i" else 0x00
        return bytes([0x10, flags, 0, 0]) + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "b":
        return bytes([0x10, 0, 0, 0]) + struct.pack("<I", 1) + struct.pack("<HH", 0, 8)
    if dt.kind == "S":
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", max(1, dt.itemsize))
    raise TypeError("unsupported dtype {}".format(dt))


def _decode_dtype(buf: bytes, off: int):
    cv = buf[off]
    cls = cv & 0x0F
    b0, b1, b2 = buf[off + 1], buf[off + 2], buf[off + 3]
    size = struct.unpack_from("<I", buf, off + 4)[0]
    bo = ">" if (b0 & 1) else "<"
    if cls == 0:
        signed = bool(b0 & 0x08)
        return np.dtype("{}{}{}".format(bo, "i" if signed else "u", size))
    if cls == 1:
        return np.dtype("{}f{}".format(bo, size))
    if cls == 3:
        return np.dtype("S{}".format(size))
    if cls == 9:
        raise NotImplementedError("variable-length types are not supported")
    raise NotImplementedError("HDF5 datatype class {}".format(cls))


def _encode_space(shape) -> bytes:
    shape = tuple(int(s) for s in shape)
    return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(struct.pack("<Q", s) for s in shape)


def _decode_space(buf: bytes, off: int):
    ver = buf[off]
    rank = buf[off + 1]
    flags = buf[off + 2]
    if ver == 1:
        p = off + 8
    elif ver == 2:
        typ = buf[off + 3]
        if typ == 0:
            return ()
        if typ == 2:
            return None
        p = off + 4
    else:
        raise NotImplementedError("dataspace version {}".format(ver))
    dims = struct.unpack_from("<{}Q".format(rank), buf, p)
    return tuple(int(d) for d in dims)


def _to_numpy_attr(value) -> np.ndarray:
    if isinstance(value, np.ndarray):
        if value.dtype.kind == "U":
            return np.char.encode(value, "utf8")
        if value.dtype.kind == "O":
            return np.array([v.encode("utf8") if isinstance(v, str) else bytes(v) for v in value.ravel()]).reshape(
                value.shape)
        return value
    if isinstance(value, str):
        return np.array(value.encode("utf8"))
    if isinstance(value, bytes):
        return np.array(value)
    if isinstance(value, (list, tuple)):
        if value and all(isinstance(v, (str, bytes)) for v in value):
            return np.array([v.encode("utf8") if isinstance(v, str) else v for v in value])
        return np.asarray(value)
    return np.asarray(value)


# =========================================================================================
# writer
# =========================================================================================
class _Writer:
    def __init__(self):
        self.buf = bytearray(b"\0" * 96)   # superblock placeholder

    def alloc(self, data: bytes, align: int = 8) -> int:
        while len(self.buf) % align:
            self.buf.append(0)
        addr = len(self.buf)
        self.buf += data
        return addr

    def reserve(self, size: int) -> int:
        return self.alloc(b"\0" * size)

    def patch(self, addr: int, data: bytes) -> None:
        self.buf[addr:addr + len(data)] = data

    @staticmethod
    def message(mtype: int, body: bytes, flags: int = 0) -> bytes:
        body = body + b"\0" * (_pad8(len(body)) - len(body))
        if len(body) > 0xFFFF:
            raise ValueError("HDF5 header message too large ({} bytes)".format(len(body)))
        return struct.pack("<HHB3x", mtype, len(body), flags) + body

    def object_header(self, messages: List[bytes]) -> int:
        body = b"".join(messages)
        hdr = struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body))
        return self.alloc(hdr + body)

    def attr_messages(self, attrs: Dict[str, Any]) -> List[bytes]:
        out = []
        for name, value in attrs.items():
            arr = _to_numpy_attr(value)
            nm = name.encode("utf8") + b"\0"
            dt = _encode_dtype(arr.dtype)
            sp = _encode_space(arr.shape)
            body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(sp))
            body += nm + b"\0" * (_pad8(len(nm)) - len(nm))
            body += dt + b"\0" * (_pad8(len(dt)) - len(dt))
            body += sp + b"\0" * (_pad8(len(sp)) - len(sp))
            body += np.ascontiguousarray(arr).astype(arr.dtype.newbyteorder("<") if arr.dtype.kind in "fiu" else
                                                     arr.dtype).tobytes()
            out.append(self.message(0x000C, body))
        return out

    def write_dataset(self, ds: Dataset) -> int:
        arr = ds._data
        if arr.dtype.kind in "fiu":
            arr = arr.astype(arr.dtype.newbyteorder("<"))
        raw = np.ascontiguousarray(arr).tobytes()
        daddr = self.alloc(raw) if raw else UNDEF
        msgs = [self.message(0x0001, _encode_space(arr.shape)),
                self.message(0x0003, _encode_dtype(arr.dtype), flags=1),
                self.message(0x0005, bytes([2, 1, 2, 0])),
                self.message(0x0008, struct.pack("<BBQQ", 3, 1, daddr, len(raw)))]
        msgs += self.attr_messages(ds.attrs)
        return self.object_header(msgs)

    def write_group(self, g: Group):
        """Returns (object header address, btree address, heap address)."""
        names = sorted(g.children.keys(), key=lambda s: s.encode("utf8"))
        child_addr = {}
        child_cache = {}
        for n in names:
            c = g.children[n]
            if isinstance(c, Group):
                oh, bt, hp = self.write_group(c)
                child_addr[n] = oh
                child_cache[n] = (bt, hp)
            else:
                child_addr[n] = self.write_dataset(c)
        # local heap: "" at offset 0, then names (8-byte padded)
        heap = bytearray(b"\0" * 8)
        offs = {}
        for n in names:
            offs[n] = len(heap)
            enc = n.encode("utf8") + b"\0"
            heap += enc + b"\0" * (_pad8(len(enc)) - len(enc))
        heap_data = self.alloc(bytes(heap))
        heap_hdr = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
        # symbol table nodes
        cap = 2 * LEAF_K
        chunks = [names[i:i + cap] for i in range(0, len(names), cap)] or [[]]
        if len(chunks) > 2 * BTREE_K:
            raise ValueError("group {} has too many members".format(g.name))
        snods = []
        for ch in chunks:
            body = b"SNOD" + struct.pack("<BBH", 1, 0, len(ch))
            for n in ch:
                if n in child_cache:
                    bt, hp = child_cache[n]
                    body += struct.pack("<QQII", offs[n], child_addr[n], 1, 0) + struct.pack("<QQ", bt, hp)
                else:
                    body += struct.pack("<QQII", offs[n], child_addr[n], 0, 0) + b"\0" * 16
            body += b"\0" * (40 * (cap - len(ch)))
            snods.append(self.alloc(body))
        # one leaf B-tree node (type 0 = group); keys = heap offsets of the last name per child
        nchild = len(snods)
        keys = [0] + [offs[ch[-1]] if ch else 0 for ch in chunks]
        body = b"TREE" + struct.pack("<BBHQQ", 0, 0, nchild if names else 0, UNDEF, UNDEF)
        for i in range(nchild if names else 0):
            body += struct.pack("<QQ", keys[i], snods[i])
        body += struct.pack("<Q", keys[nchild] if names else 0)
        full = 24 + (2 * BTREE_K + 1) * 8 + 2 * BTREE_K * 8
        body += b"\0" * (full - len(body))
        btree = self.alloc(body)
        msgs = [self.message(0x0011, struct.pack("<QQ", btree, heap_hdr))]
        msgs += self.attr_messages(g.attrs)
        oh = self.object_header(msgs)
        return oh, btree, heap_hdr

    def finish(self, root: Group) -> bytes:
        oh, bt, hp = self.write_group(root)
        eof = len(self.buf)
        sb = SIG + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0)
        sb += struct.pack("<HHI", LEAF_K, BTREE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", bt, hp)
        assert len(sb) == 96
        self.patch(0, sb)
        return bytes(self.buf)


# =========================================================================================
# reader
# =========================================================================================
class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        if data[:8] != SIG:
            raise ValueError("not an HDF5 file")
        ver = data[8]
        if ver in (0, 1):
            self.so = data[13]
            self.sl = data[14]
            p = 24 if ver == 0 else 28
            p += 4 * 8
            self.root_oh = struct.unpack_from("<Q", data, p + 8)[0]
        elif ver in (2, 3):
            self.so, self.sl = data[9], data[10]
            self.root_oh = struct.unpack_from("<Q", data, 12 + 3 * 8)[0]
        else:
            raise NotImplementedError("superblock version {}".format(ver))

    def _q(self, off):
        return struct.unpack_from("<Q", self.d, off)[0]

    def messages(self, addr: int):
        d = self.d
        if d[addr:addr + 4] == b"OHDR":
            return list(self._messages_v2(addr))
        ver = d[addr]
        if ver != 1:
            raise NotImplementedError("object header version {}".format(ver))
        nmsg = struct.unpack_from("<H", d, addr + 2)[0]
        size = struct.unpack_from("<I", d, addr + 8)[0]
        blocks = [(addr + 16, size)]
        out = []
        while blocks and len(out) < nmsg:
            p, sz = blocks.pop(0)
            end = p + sz
            while p + 8 <= end and len(out) < nmsg:
                mtype, msz, flags = struct.unpack_from("<HHB", d, p)
                body = d[p + 8:p + 8 + msz]
                if mtype == 0x0010:
                    caddr, clen = struct.unpack_from("<QQ", body, 0)
                    blocks.append((caddr, clen))
                out.append((mtype, body))
                p += 8 + msz
        return out

    def _messages_v2(self, addr):
        d = self.d
        flags = d[addr + 5]
        p = addr + 6
        if flags & 0x20:
            p += 16
        if flags & 0x10:
            p += 4
        szb = 1 << (flags & 3)
        size = int.from_bytes(d[p:p + szb], "little")
        p += szb
        blocks = [(p, size, True)]
        while blocks:
            start, sz, first = blocks.pop(0)
            q = start
            end = start + sz
            while q + 4 <= end:
                mtype = d[q]
                msz = struct.unpack_from("<H", d, q + 1)[0]
                mflags = d[q + 3]
                q += 4
                if flags & 0x04:
                    q += 2
                body = d[q:q + msz]
                if mtype == 0x10:
                    caddr, clen = struct.unpack_from("<QQ", body, 0)
                    blocks.append((caddr + 4, clen - 8, False))
                yield (mtype, body)
                q += msz

    def _attr(self, body: bytes):
        ver = body[0]
        if ver == 1:
            nsz, dsz, ssz = struct.unpack_from("<HHH", body, 2)
            p = 8
            name = body[p:p + nsz].split(b"\0")[0].decode("utf8")
            p += _pad8(nsz)
            dt = _decode_dtype(body, p)
            p += _pad8(dsz)
            shape = _decode_space(body, p)
            p += _pad8(ssz)
        elif ver in (2, 3):
            nsz, dsz, ssz = struct.unpack_from("<HHH", body, 2)
            p = 8 + (1 if ver == 3 else 0)
            name = body[p:p + nsz].split(b"\0")[0].decode("utf8")
            p += nsz
            dt = _decode_dtype(body, p)
            p += dsz
            shape = _decode_space(body, p)
            p += ssz
        else:
            raise NotImplementedError("attribute message version {}".format(ver))
        n = int(np.prod(shape)) if shape else 1
        arr = np.frombuffer(body, dtype=dt, count=n, offset=p).reshape(shape if shape else ())
        return name, arr.copy()

    def read_object(self, addr: int, name: str):
        msgs = self.messages(addr)
        types = [m[0] for m in msgs]
        attrs = Attrs()
        for t, b in msgs:
            if t == 0x000C:
                k, v = self._attr(b)
                attrs[k] = v
        if 0x0011 in types:
            g = Group(name)
            g.attrs = attrs
            body = msgs[types.index(0x0011)][1]
            bt, hp = struct.unpack_from("<QQ", body, 0)
            heap_data = self._q(hp + 24)
            for off, oh in self._btree_entries(bt):
                nm = self.d[heap_data + off:self.d.index(b"\0", heap_data + off)].decode("utf8")
                g.children[nm] = self.read_object(oh, name.rstrip("/") + "/" + nm)
            return g
        if 0x0006 in types or 0x0002 in types:
            g = Group(name)
            g.attrs = attrs
            for t, b in msgs:
                if t == 0x0006:
                    nm, oh = self._link(b)
                    if oh is not None:
                        g.children[nm] = self.read_object(oh, name.rstrip("/") + "/" + nm)
            return g
        shape = dt = None
        layout = None
        for t, b in msgs:
            if t == 0x0001:
                shape = _decode_space(b, 0)
            elif t == 0x0003:
                dt = _decode_dtype(b, 0)
            elif t == 0x0008:
                layout = b
        data = self._layout_data(layout, shape, dt)
        return Dataset(name, data, attrs)

    def _link(self, b: bytes):
        flags = b[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = b[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        lsz = 1 << (flags & 3)
        nlen = int.from_bytes(b[p:p + lsz], "little")
        p += lsz
        nm = b[p:p + nlen].decode("utf8")
        p += nlen
        if ltype != 0:
            return nm, None
        return nm, struct.unpack_from("<Q", b, p)[0]

    def _btree_entries(self, addr: int):
        d = self.d
        if d[addr:addr + 4] != b"TREE":
            raise ValueError("bad B-tree signature")
        level = d[addr + 5]
        n = struct.unpack_from("<H", d, addr + 6)[0]
        p = addr + 24
        children = []
        for i in range(n):
            p += 8
            children.append(self._q(p))
            p += 8
        out = []
        for c in children:
            if level > 0:
                out.extend(self._btree_entries(c))
            else:
                if d[c:c + 4] != b"SNOD":
                    raise ValueError("bad symbol node")
                cnt = struct.unpack_from("<H", d, c + 6)[0]
                for j in range(cnt):
                    e = c + 8 + 40 * j
                    out.append((self._q(e), self._q(e + 8)))
        return out

    def _layout_data(self, b: bytes, shape, dt):
        if shape is None:
            return np.zeros((0,), dtype=dt)
        n = int(np.prod(shape)) if shape else 1
        ver = b[0]
        if ver == 3:
            cls = b[1]
            if cls == 0:
                sz = struct.unpack_from("<H", b, 2)[0]
                raw = b[4:4 + sz]
            elif cls == 1:
                addr, sz = struct.unpack_from("<QQ", b, 2)
                raw = self.d[addr:addr + sz] if addr != UNDEF else b"\0" * (n * dt.itemsize)
            else:
                raise NotImplementedError("chunked datasets are not supported")
        elif ver in (1, 2):
            rank = b[1]
            cls = b[2]
            if cls != 1:
                raise NotImplementedError("layout class {}".format(cls))
            addr = struct.unpack_from("<Q", b, 8)[0]
            raw = self.d[addr:addr + n * dt.itemsize]
        else:
            raise NotImplementedError("layout version {}".format(ver))
        return np.frombuffer(raw, dtype=dt, count=n).reshape(shape).copy()

    def root(self) -> Group:
        return self.read_object(self.root_oh, "/")


# =========================================================================================
# h5py-like file object
# =========================================================================================
class File(Group):
    def __init__(self, path: str, mode: str = "r"):
        super().__init__("/")
        self.path = path
        self.mode = mode
        if mode == "r":
            with open(path, "rb") as f:
                g = _Reader(f.read()).root()
            self.attrs, self.children = g.attrs, g.children
        elif mode not in ("w", "x"):
            raise ValueError("mode must be 'r' or 'w'")

    def close(self) -> None:
        if self.mode in ("w", "x"):
            data = _Writer().finish(self)
            tmp = self.path + ".tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, self.path)
            self.mode = "closed"

    def flush(self) -> None:
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def save_attributes_to_hdf5_group(group: Group, name: str, data, limit: int = 64512) -> None:
    """Keras' chunking of big attributes (``name0``, ``name1``, ...) to fit header messages."""
    arr = _to_numpy_attr(data)
    if arr.nbytes <= limit:
        group.attrs[name] = arr
        return
    n = int(np.ceil(arr.nbytes / limit))
    chunks = np.array_split(arr, n) if arr.ndim else [arr]
    while any(c.nbytes > limit for c in chunks):
        n += 1
        chunks = np.array_split(arr, n)
    for i, c in enumerate(chunks):
        group.attrs["%s%d" % (name, i)] = c


def load_attributes_from_hdf5_group(group: Group, name: str):
    if name in group.attrs:
        v = group.attrs[name]
        return [x.decode("utf8") for x in np.atleast_1d(v)] if v.dtype.kind == "S" else v
    out, i = [], 0
    while "%s%d" % (name, i) in group.attrs:
        v = group.attrs["%s%d" % (name, i)]
        out.extend([x.decode("utf8") for x in np.atleast_1d(v)])
        i += 1
    return out
