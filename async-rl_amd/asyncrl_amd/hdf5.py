"""Chainer-HDF5 checkpoints without h5py.

The reference saves and loads its model and optimizer with
`chainer.serializers.save_hdf5` / `load_hdf5` (a3c.py:169-185,
demo_a3c_ale.py:61).  Those files are HDF5 1.8-era files written by h5py:
superblock version 0, version-1 object headers, groups as symbol tables
(v1 B-tree + local heap + symbol nodes), datasets chunked and deflated
(compression=4) or contiguous.  h5py is not a dependency here, so this
module reads and writes exactly that subset with the standard library and
NumPy:

  read_hdf5(path)  -> {"0/0/W": ndarray, ...}   (every dataset, by path)
  write_hdf5(path, {"0/0/W": ndarray, ...})      (groups from the paths;
                                                  contiguous datasets)

Supported on read: superblock v0/v1 with 8-byte offsets and lengths, object
header v1 (+ continuation blocks), symbol-table groups, dataspace v1/v2,
fixed-point / IEEE-float datatypes (either byte order), layout message v3
(compact, contiguous, chunked with a v1 chunk B-tree), filters deflate and
shuffle.  Anything else raises ValueError naming what was found.  Host-side
setup code, not on the hot path.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"
_UNDEF = 0xFFFFFFFFFFFFFFFF


# ---------------------------------------------------------------------------- read
class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        if data[:8] != _SIG:
            raise ValueError("not an HDF5 file (signature)")
        ver = data[8]
        if ver not in (0, 1):
            raise ValueError("HDF5 superblock version %d not supported (0/1 only)" % ver)
        if data[13] != 8 or data[14] != 8:
            raise ValueError("HDF5 offsets/lengths must be 8 bytes")
        p = 24 if ver == 0 else 28
        self.base = struct.unpack_from("<Q", data, p)[0]
        root = p + 32                       # base, free-space, eof, driver addresses
        self.root = struct.unpack_from("<Q", data, root + 8)[0]

    def u(self, fmt, off):
        return struct.unpack_from("<" + fmt, self.d, off)

    # object header v1 -> list of (type, body bytes)
    def messages(self, addr):
        d = self.d
        if d[addr] != 1:
            raise ValueError("object header version %d at %d not supported" % (d[addr], addr))
        nmsg, _, hsize = self.u("HII", addr + 2)
        blocks = [(addr + 16, hsize)]
        out = []
        while blocks:
            p, size = blocks.pop(0)
            end = p + size
            while p + 8 <= end and len(out) < nmsg:
                mtype, msize = self.u("HH", p)
                body = d[p + 8:p + 8 + msize]
                out.append((mtype, body))
                if mtype == 0x10:           # continuation
                    caddr, clen = struct.unpack_from("<QQ", body, 0)
                    blocks.append((caddr, clen))
                p += 8 + msize
        return out

    def children(self, btree, heap):
        """(name, object header address) of a symbol-table group."""
        d = self.d
        if d[heap:heap + 4] != b"HEAP":
            raise ValueError("local heap signature")
        heap_data = self.u("Q", heap + 24)[0]
        out = []

        def name_at(off):
            s = heap_data + off
            return d[s:d.index(b"\0", s)].decode()

        def walk(node):
            if d[node:node + 4] != b"TREE":
                raise ValueError("group B-tree signature")
            ntype, level, used = d[node + 4], d[node + 5], self.u("H", node + 6)[0]
            if ntype != 0:
                raise ValueError("group B-tree node type %d" % ntype)
            p = node + 24 + 8                  # skip key 0
            for _ in range(used):
                child = self.u("Q", p)[0]
                p += 16                        # child + next key
                if level > 0:
                    walk(child)
                else:
                    if d[child:child + 4] != b"SNOD":
                        raise ValueError("symbol node signature")
                    nsym = self.u("H", child + 6)[0]
                    for i in range(nsym):
                        e = child + 8 + 40 * i
                        noff, oh = self.u("QQ", e)
                        out.append((name_at(noff), oh))
        walk(btree)
        return out

    @staticmethod
    def dtype(body):
        cls_ver = body[0]
        cls = cls_ver & 0x0F
        bits = body[1]
        size = struct.unpack_from("<I", body, 4)[0]
        order = ">" if bits & 1 else "<"
        if cls == 0:
            signed = bool(bits & 0x08)
            return np.dtype(order + ("i" if signed else "u") + str(size))
        if cls == 1:
            if size not in (2, 4, 8):
                raise ValueError("float size %d" % size)
            return np.dtype(order + "f" + str(size))
        raise ValueError("HDF5 datatype class %d not supported" % cls)

    @staticmethod
    def dataspace(body):
        ver, rank, flags = body[0], body[1], body[2]
        p = 8 if ver == 1 else 4
        if ver == 2 and body[3] == 2:          # null dataspace
            return None
        return tuple(struct.unpack_from("<%dQ" % rank, body, p)) if rank else ()

    @staticmethod
    def filters(body):
        ver, n = body[0], body[1]
        p = 8 if ver == 1 else 2
        out = []
        for _ in range(n):
            fid, = struct.unpack_from("<H", body, p)
            if ver == 1 or fid >= 256:
                nlen, flags, nval = struct.unpack_from("<HHH", body, p + 2)
                p += 8
                p += (nlen + 7) // 8 * 8 if ver == 1 else nlen
            else:
                flags, nval = struct.unpack_from("<HH", body, p + 2)
                p += 6
            vals = struct.unpack_from("<%dI" % nval, body, p)
            p += 4 * nval
            if ver == 1 and nval % 2:
                p += 4
            out.append((fid, vals))
        return out

    def dataset(self, msgs):
        shape = dt = layout = None
        filt = []
        for t, b in msgs:
            if t == 0x01:
                shape = self.dataspace(b)
            elif t == 0x03:
                dt = self.dtype(b)
            elif t == 0x08:
                layout = b
            elif t == 0x0B:
                filt = self.filters(b)
        if shape is None or dt is None or layout is None:
            raise ValueError("dataset without dataspace / datatype / layout")
        if layout[0] != 3:
            raise ValueError("data layout message version %d not supported (3 only)" % layout[0])
        lclass = layout[1]
        n = int(np.prod(shape)) if shape else 1
        nbytes = n * dt.itemsize
        if lclass == 0:                         # compact
            size, = struct.unpack_from("<H", layout, 2)
            raw = layout[4:4 + size]
            return np.frombuffer(raw, dt, n).reshape(shape).astype(dt.newbyteorder("="))
        if lclass == 1:                         # contiguous
            addr, size = struct.unpack_from("<QQ", layout, 2)
            if addr == _UNDEF:
                return np.zeros(shape, dt.newbyteorder("="))
            raw = self.d[addr:addr + nbytes]
            return np.frombuffer(raw, dt, n).reshape(shape).astype(dt.newbyteorder("="))
        if lclass != 2:
            raise ValueError("layout class %d" % lclass)
        rank1 = layout[2]
        btree, = struct.unpack_from("<Q", layout, 3)
        cdims = struct.unpack_from("<%dI" % rank1, layout, 11)[:-1]
        out = np.zeros(shape, dt)
        if btree == _UNDEF:
            return out.astype(dt.newbyteorder("="))
        for off, size, mask, addr in self._chunks(btree, rank1):
            raw = self.d[addr:addr + size]
            for i, (fid, vals) in reversed(list(enumerate(filt))):
                if mask & (1 << i):
                    continue
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:                  # shuffle: bytes were grouped by significance
                    es = vals[0] if vals else dt.itemsize
                    a = np.frombuffer(raw, np.uint8)
                    m = len(a) // es
                    raw = a[:m * es].reshape(es, m).T.tobytes() + a[m * es:].tobytes()
                else:
                    raise ValueError("HDF5 filter %d not supported" % fid)
            chunk = np.frombuffer(raw, dt, int(np.prod(cdims))).reshape(cdims)
            sl_out = tuple(slice(o, min(o + c, s)) for o, c, s in zip(off, cdims, shape))
            sl_in = tuple(slice(0, s.stop - s.start) for s in sl_out)
            out[sl_out] = chunk[sl_in]
        return out.astype(dt.newbyteorder("="))

    def _chunks(self, node, rank1):
        d = self.d
        if d[node:node + 4] != b"TREE" or d[node + 4] != 1:
            raise ValueError("chunk B-tree signature / type")
        level, used = d[node + 5], self.u("H", node + 6)[0]
        ksize = 8 + 8 * rank1
        p = node + 24
        out = []
        for _ in range(used):
            size, mask = self.u("II", p)
            off = self.u("%dQ" % (rank1 - 1), p + 8)
            child, = self.u("Q", p + ksize)
            if level > 0:
                out += self._chunks(child, rank1)
            else:
                out.append((off, size, mask, child))
            p += ksize + 8
        return out

    def walk(self, addr, prefix, out):
        msgs = self.messages(addr)
        stab = [b for t, b in msgs if t == 0x11]
        if stab:
            btree, heap = struct.unpack_from("<QQ", stab[0], 0)
            for name, child in self.children(btree, heap):
                self.walk(child, prefix + name + "/", out)
        elif any(t == 0x08 for t, _ in msgs):
            out[prefix[:-1]] = self.dataset(msgs)
        elif any(t in (0x02, 0x0A) for t, _ in msgs):
            raise ValueError("new-style (link message) groups not supported")
        return out


def read_hdf5(path) -> dict:
    """Every dataset of a Chainer/h5py HDF5 file, keyed by its path
    ("0/0/W"), as native-byte-order NumPy arrays."""
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    return r.walk(r.root, "", {})


# ---------------------------------------------------------------------------- write
_GROUP_LEAF_K = 4          # symbol node holds 2K entries (superblock field)
_GROUP_INTERNAL_K = 16     # group B-tree node holds up to 2K children


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


def _msg(mtype: int, body: bytes, flags: int = 0) -> bytes:
    body = _pad8(body)
    return struct.pack("<HHB3x", mtype, len(body), flags) + body


def _ohdr(msgs) -> bytes:
    body = b"".join(msgs)
    return struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body)) + body


def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt).newbyteorder("<")
    if dt.kind == "f":
        sign, prec, eloc, esz, msz, bias = {2: (15, 16, 10, 5, 10, 15), 4: (31, 32, 23, 8, 23, 127),
                                            8: (63, 64, 52, 11, 52, 1023)}[dt.itemsize]
        return struct.pack("<BBBBI", 0x11, 0x20, sign, 0, dt.itemsize) + \
            struct.pack("<HHBBBBI", 0, prec, eloc, esz, 0, msz, bias)
    if dt.kind in "iub":
        signed = 0x08 if dt.kind == "i" else 0
        return struct.pack("<BBBBI", 0x10, signed, 0, 0, dt.itemsize) + struct.pack("<HH", 0, 8 * dt.itemsize)
    raise ValueError("dtype %s not writable" % dt)


class _Writer:
    def __init__(self):
        self.buf = bytearray(b"\0" * 96)      # superblock + root symbol table entry, patched last

    def put(self, b: bytes) -> int:
        addr = len(self.buf)
        self.buf += _pad8(b)
        return addr

    def dataset(self, a: np.ndarray) -> int:
        a = np.asarray(a)                      # (keeps 0-d: scalars such as the optimizer's t)
        if not a.flags.c_contiguous:
            a = a.copy(order="C")
        if a.dtype == np.bool_:
            a = a.astype(np.uint8)
        a = a.astype(a.dtype.newbyteorder("<"), copy=False)
        data_addr = self.put(a.tobytes()) if a.nbytes else _UNDEF
        space = struct.pack("<BBB5x", 1, a.ndim, 0) + b"".join(struct.pack("<Q", s) for s in a.shape)
        fill = struct.pack("<BBBB", 2, 1, 2, 0)            # v2: early alloc, fill never, undefined
        layout = struct.pack("<BBQQ", 3, 1, data_addr, a.nbytes)
        return self.put(_ohdr([_msg(0x01, space), _msg(0x03, _dtype_msg(a.dtype)), _msg(0x05, fill, 1),
                               _msg(0x08, layout)]))

    def group(self, tree: dict):
        """Returns (object header address, B-tree address, heap address)."""
        entries = []
        for name in sorted(tree):
            v = tree[name]
            if isinstance(v, dict):
                oh, bt, hp = self.group(v)
                entries.append((name, oh, 1, bt, hp))
            else:
                entries.append((name, self.dataset(v), 0, 0, 0))
        # local heap: "" at offset 0, then the names
        heap = bytearray(b"\0" * 8)
        noff = {}
        for name, *_ in entries:
            noff[name] = len(heap)
            heap += _pad8(name.encode() + b"\0")
        heap_data = self.put(bytes(heap))
        # free-list head 1 = H5HL_FREE_NULL (the segment is exactly full)
        heap_addr = self.put(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
        # symbol nodes (2K entries each, full size allocated)
        cap = 2 * _GROUP_LEAF_K
        snods = []
        for i in range(0, max(len(entries), 1), cap):
            part = entries[i:i + cap]
            b = bytearray(b"SNOD" + struct.pack("<BBH", 1, 0, len(part)))
            for name, oh, ctype, bt, hp in part:
                scratch = struct.pack("<QQ", bt, hp) if ctype == 1 else b"\0" * 16
                b += struct.pack("<QQI4x", noff[name], oh, ctype) + scratch
            b += b"\0" * (8 + 40 * cap - len(b))
            snods.append((self.put(bytes(b)), noff[part[-1][0]] if part else 0))
        if len(snods) > 2 * _GROUP_INTERNAL_K:
            raise ValueError("group too large for a single B-tree node")
        # B-tree (type 0, leaf level): key0 = 0, child, key(last name of the node), ...
        bt = bytearray(b"TREE" + struct.pack("<BBHQQ", 0, 0, len(snods), _UNDEF, _UNDEF))
        bt += struct.pack("<Q", 0)
        for addr, lastkey in snods:
            bt += struct.pack("<QQ", addr, lastkey)
        full = 24 + 8 * (2 * _GROUP_INTERNAL_K + 1) + 8 * 2 * _GROUP_INTERNAL_K
        bt += b"\0" * (full - len(bt))
        bt_addr = self.put(bytes(bt))
        oh = self.put(_ohdr([_msg(0x11, struct.pack("<QQ", bt_addr, heap_addr))]))
        return oh, bt_addr, heap_addr

    def finish(self, root) -> bytes:
        oh, bt, hp = root
        sb = _SIG + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0)
        sb += struct.pack("<HHI", _GROUP_LEAF_K, _GROUP_INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, _UNDEF, len(self.buf), _UNDEF)
        sb += struct.pack("<QQI4xQQ", 0, oh, 1, bt, hp)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def write_hdf5(path, arrays: dict) -> None:
    """Write {path: ndarray} as an HDF5 file with the group structure the
    paths imply ("0/0/W" -> group 0, group 0/0, dataset W), readable by
    h5py / chainer.serializers.load_hdf5 and by read_hdf5."""
    tree: dict = {}
    for key, val in arrays.items():
        parts = [p for p in key.split("/") if p]
        node = tree
        for p in parts[:-1]:
            node = node.setdefault(p, {})
            if not isinstance(node, dict):
                raise ValueError("path %s crosses a dataset" % key)
        node[parts[-1]] = np.asarray(val)
    w = _Writer()
    data = w.finish(w.group(tree))
    with open(path, "wb") as f:
        f.write(data)
