"""Self-describing wire format of a compressed update ("COALAQ1").

The blob rides inside the pickled carrier that COALA puts into UploadContent.data
(/root/reference/coala/client/base.py:363 -> protos/coala/pb/server_service.proto:13-24). It must be
self-describing because remote clients never receive new config keys (OperateConfig has fixed fields,
/root/reference/protos/coala/pb/client_service.proto:24-39).

Layout (little-endian):
    0   8B   magic b"COALAQ1\\0"
    8   u32  format version (2 when the header has "n_units", else 1)
    12  u32  header length H
    16  H    UTF-8 JSON header: ratio, bits, mode, n_segments, total_k, [n_units], entries[]
             entry = {"name", "dtype", "shape", "kind": "seg", "seg": i, "n", "k", "out_off"}
                   | {"name", "dtype", "shape", "kind": "raw", "off", "nbytes"}
    then, each section starting at a 16-byte boundary:
         mn f32[T] | scale f32[T] | idx i32[K] | vals (u8[K], or f32[K] if bits == 32) | [ustart i32[U]] | raw bytes
    ustart (version 2): per 4096-element unit of every fp32 segment, in segment order, the segment-relative
    index of the unit's first kept entry — what the encoder's k_select computed anyway, so the decoder (and the
    server's fused aggregate) finds each unit's entries without searching the idx lists. U = "n_units".
    A header with "dense": true (ratio 1: every segment keeps all n elements, idx = 0..n-1 per segment)
    carries an empty idx section, and unpack returns an empty idx: the indices stay implied all the way into
    the GPU's dense decode (coalac.hip k_dense_deq), never materialised. This is the download-direction
    default (dense 8-bit weights, ~4x smaller than fp32 instead of 5 B per element with explicit indices).
"""
import json
import struct
import threading
from collections import OrderedDict

import numpy as np

MAGIC = b"COALAQ1\0"
VERSION = 1     # mn | scale | idx | vals | raw
VERSION_2 = 2   # ... | vals | ustart | raw


def _pad16(n):
    return (16 - n % 16) % 16


def pack(header, mn, scale, idx, vals, raw, header_json=None, ustart=None):
    """numpy arrays + raw bytes -> blob (bytes). A "dense" header drops idx (it is implied). header_json: the
    header's JSON encoding, if the caller has it already. ustart: the per-unit starts (version 2; the header
    must then carry "n_units" = len(ustart))."""
    if header.get("dense"):
        idx = np.zeros(0, dtype=np.int32)
    if (ustart is not None) != ("n_units" in header) or (ustart is not None and len(ustart) != header["n_units"]):
        raise ValueError("COALAQ1: ustart section and header n_units disagree")
    h = header_json if header_json is not None else encode_header(header)
    parts = [MAGIC, struct.pack("<II", VERSION if ustart is None else VERSION_2, len(h)), h]
    size = 16 + len(h)
    arrays = [np.ascontiguousarray(mn, "<f4"), np.ascontiguousarray(scale, "<f4"),
              np.ascontiguousarray(idx, "<i4"), np.ascontiguousarray(vals)]
    if ustart is not None:
        arrays.append(np.ascontiguousarray(ustart, "<i4"))
    for arr in arrays:
        p = _pad16(size)
        parts.append(b"\0" * p)
        b = arr.tobytes()
        parts.append(b)
        size += p + len(b)
    p = _pad16(size)
    parts.append(b"\0" * p)
    parts.append(bytes(raw))
    return b"".join(parts)


_HEADERS = OrderedDict()  # header JSON bytes -> parsed header (the same layout arrives round after round)
_HEADERS_LOCK = threading.Lock()


def _parse_header(mv, hl):
    """The blob's JSON header, parsed once per distinct header text (LRU of 32): a SHALLOW copy of the
    cached dict is returned — its "entries" list is shared and must never be mutated (nothing does)."""
    key = bytes(mv[16:16 + hl])
    with _HEADERS_LOCK:
        h = _HEADERS.get(key)
        if h is not None:
            _HEADERS.move_to_end(key)
    if h is None:
        h = json.loads(key.decode())
        with _HEADERS_LOCK:
            _HEADERS[key] = h
            while len(_HEADERS) > 32:
                _HEADERS.popitem(last=False)
    return dict(h)


def encode_header(header):
    return json.dumps(header, separators=(",", ":"), sort_keys=True).encode()


def sections(blob, header=None):
    """(header, {name: (byte offset, byte count)}) of the mn / scale / idx / vals (/ ustart) sections in `blob`,
    which lie back to back (each 16-byte aligned) — one host-to-device copy moves all of them."""
    mv = memoryview(blob)
    if bytes(mv[:8]) != MAGIC:
        raise ValueError("not a COALAQ1 blob (bad magic)")
    ver, hl = struct.unpack_from("<II", mv, 8)
    if header is None:
        header = _parse_header(mv, hl)
    T, K = int(header["n_segments"]), int(header["total_k"])
    vsz = 4 if int(header["bits"]) == 32 else 1
    pos = 16 + hl
    out = {}
    names = [("mn", 4 * T), ("scale", 4 * T), ("idx", 0 if header.get("dense") else 4 * K), ("vals", vsz * K)]
    if "n_units" in header:
        names.append(("ustart", 4 * int(header["n_units"])))
    for name, n in names:
        pos += _pad16(pos)
        out[name] = (pos, n)
        pos += n
    return header, out


def unpack(blob):
    """blob -> (header dict, mn, scale, idx, vals, raw bytes, ustart or None). Arrays are read-only views of
    blob; a "dense" blob's idx is empty (implied)."""
    mv = memoryview(blob)
    if bytes(mv[:8]) != MAGIC:
        raise ValueError("not a COALAQ1 blob (bad magic)")
    ver, hl = struct.unpack_from("<II", mv, 8)
    if ver not in (VERSION, VERSION_2):
        raise ValueError(f"unsupported COALAQ1 version {ver}")
    header = _parse_header(mv, hl)
    if (ver == VERSION_2) != ("n_units" in header):
        raise ValueError("COALAQ1: version and header n_units disagree")
    T, K = int(header["n_segments"]), int(header["total_k"])
    vdt = np.dtype("<f4") if int(header["bits"]) == 32 else np.dtype("u1")
    pos = 16 + hl
    out = []
    dense = bool(header.get("dense"))
    layout = [(np.dtype("<f4"), T), (np.dtype("<f4"), T), (np.dtype("<i4"), 0 if dense else K), (vdt, K)]
    if ver == VERSION_2:
        layout.append((np.dtype("<i4"), int(header["n_units"])))
    for dt, n in layout:
        pos += _pad16(pos)
        if n < 0 or pos + n * dt.itemsize > len(mv):
            raise ValueError("COALAQ1: truncated blob")
        out.append(np.frombuffer(mv, dtype=dt, count=n, offset=pos))
        pos += n * dt.itemsize
    pos += _pad16(pos)
    raw = bytes(mv[pos:])
    if dense and K != sum(int(e["n"]) for e in header["entries"] if e["kind"] == "seg"):
        raise ValueError("COALAQ1: dense header with k != n")
    ustart = out[4] if ver == VERSION_2 else None
    return (header, *out[:4], raw, ustart)
