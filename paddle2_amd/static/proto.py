"""Protocol-buffer wire codec for the reference's ProgramDesc schema (paddle/fluid/framework/framework.proto),
and the LoDTensor stream format of ``.pdiparams`` (lod_tensor.cc SerializeToStream, tensor_util.cc
TensorToStream).

No protoc / generated classes: a message is a plain dict, described by a small schema table of
(field number -> name, wire kind, repeated, sub-message).  Enough of proto2 for these files: varints
(int32/int64/bool/enum, negative int64 as 10-byte two's complement), fixed32 float, fixed64 double,
length-delimited strings / bytes / sub-messages, packed or unpacked repeated scalars on read.
"""
from __future__ import annotations

import struct

# (name, kind, repeated, submessage) ; kind in {"varint", "sint?"(unused), "float", "double", "string", "bytes", "msg"}
SCHEMA = {
    "Version": {1: ("version", "varint", False, None)},
    "Complex": {1: ("r", "double", False, None), 2: ("i", "double", False, None)},
    "Scalar": {1: ("type", "varint", False, None), 2: ("b", "varint", False, None), 3: ("i", "varint", False, None),
               4: ("r", "double", False, None), 5: ("c", "msg", False, "Complex")},
    "OpDesc.Attr": {
        1: ("name", "string", False, None), 2: ("type", "varint", False, None), 3: ("i", "varint", False, None),
        4: ("f", "float", False, None), 5: ("s", "string", False, None), 6: ("ints", "varint", True, None),
        7: ("floats", "float", True, None), 8: ("strings", "string", True, None), 10: ("b", "varint", False, None),
        11: ("bools", "varint", True, None), 12: ("block_idx", "varint", False, None),
        13: ("l", "varint", False, None), 14: ("blocks_idx", "varint", True, None),
        15: ("longs", "varint", True, None), 16: ("float64s", "double", True, None),
        17: ("var_name", "string", False, None), 18: ("vars_name", "string", True, None),
        19: ("float64", "double", False, None), 20: ("scalar", "msg", False, "Scalar"),
        21: ("scalars", "msg", True, "Scalar")},
    "OpDesc.Var": {1: ("parameter", "string", False, None), 2: ("arguments", "string", True, None)},
    "OpDesc": {3: ("type", "string", False, None), 1: ("inputs", "msg", True, "OpDesc.Var"),
               2: ("outputs", "msg", True, "OpDesc.Var"), 4: ("attrs", "msg", True, "OpDesc.Attr"),
               5: ("is_target", "varint", False, None)},
    "TensorDesc": {1: ("data_type", "varint", False, None), 2: ("dims", "varint", True, None)},
    "LoDTensorDesc": {1: ("tensor", "msg", False, "TensorDesc"), 2: ("lod_level", "varint", False, None)},
    "VarType": {1: ("type", "varint", False, None), 2: ("selected_rows", "msg", False, "TensorDesc"),
                3: ("lod_tensor", "msg", False, "LoDTensorDesc"), 4: ("tensor_array", "msg", False, "LoDTensorDesc")},
    "VarDesc.Attr": {1: ("name", "string", False, None), 2: ("type", "varint", False, None),
                     3: ("i", "varint", False, None), 4: ("s", "string", False, None),
                     5: ("ints", "varint", True, None)},
    "VarDesc": {1: ("name", "string", False, None), 2: ("type", "msg", False, "VarType"),
                3: ("persistable", "varint", False, None), 4: ("need_check_feed", "varint", False, None),
                5: ("is_parameter", "varint", False, None), 6: ("stop_gradient", "varint", False, None),
                7: ("attrs", "msg", True, "VarDesc.Attr")},
    "BlockDesc": {1: ("idx", "varint", False, None), 2: ("parent_idx", "varint", False, None),
                  3: ("vars", "msg", True, "VarDesc"), 4: ("ops", "msg", True, "OpDesc"),
                  5: ("forward_block_idx", "varint", False, None)},
    "OpVersion": {1: ("version", "varint", False, None)},
    "OpVersionPair": {1: ("op_name", "string", False, None), 2: ("op_version", "msg", False, "OpVersion")},
    "OpVersionMap": {1: ("pair", "msg", True, "OpVersionPair")},
    "ProgramDesc": {1: ("blocks", "msg", True, "BlockDesc"), 4: ("version", "msg", False, "Version"),
                    5: ("op_version_map", "msg", False, "OpVersionMap")},
}
_BY_NAME = {m: {v[0]: (k,) + v[1:] for k, v in f.items()} for m, f in SCHEMA.items()}

# VarType.Type / AttrType enums
VT = {"BOOL": 0, "INT16": 1, "INT32": 2, "INT64": 3, "FP16": 4, "FP32": 5, "FP64": 6, "LOD_TENSOR": 7,
      "FEED_MINIBATCH": 9, "FETCH_LIST": 10, "UINT8": 20, "INT8": 21, "BF16": 22, "COMPLEX64": 23, "COMPLEX128": 24}
AT = {"INT": 0, "FLOAT": 1, "STRING": 2, "INTS": 3, "FLOATS": 4, "STRINGS": 5, "BOOLEAN": 6, "BOOLEANS": 7,
      "BLOCK": 8, "LONG": 9, "BLOCKS": 10, "LONGS": 11, "FLOAT64S": 12, "VAR": 13, "VARS": 14, "FLOAT64": 15}


# ------------------------------------------------------------------------------------------- wire level
def _varint(v):
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, i):
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def _signed(v, bits=64):
    return v - (1 << 64) if v >= 1 << 63 else v


def encode(msg, name):
    fields = _BY_NAME[name]
    out = bytearray()
    # field-number order (deterministic, what a C++ SerializeAsString produces)
    for fname, (num, kind, rep, sub) in sorted(fields.items(), key=lambda kv: kv[1][0]):
        if fname not in msg or msg[fname] is None:
            continue
        vals = msg[fname] if rep else [msg[fname]]
        for v in vals:
            if kind == "varint":
                out += _varint(num << 3) + _varint(int(v))
            elif kind == "float":
                out += _varint((num << 3) | 5) + struct.pack("<f", float(v))
            elif kind == "double":
                out += _varint((num << 3) | 1) + struct.pack("<d", float(v))
            elif kind in ("string", "bytes"):
                b = v.encode() if isinstance(v, str) else bytes(v)
                out += _varint((num << 3) | 2) + _varint(len(b)) + b
            else:
                b = encode(v, sub)
                out += _varint((num << 3) | 2) + _varint(len(b)) + b
    return bytes(out)


def decode(buf, name, i=0, end=None):
    fields = SCHEMA[name]
    end = len(buf) if end is None else end
    msg = {}
    for num, (fname, kind, rep, sub) in fields.items():
        if rep:
            msg[fname] = []
    while i < end:
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        spec = fields.get(num)
        if wt == 0:
            v, i = _read_varint(buf, i)
            val = _signed(v)
        elif wt == 1:
            val = struct.unpack_from("<d", buf, i)[0] if (spec and spec[1] == "double") else struct.unpack_from(
                "<q", buf, i)[0]
            i += 8
        elif wt == 5:
            val = struct.unpack_from("<f", buf, i)[0]
            i += 4
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            j = i + ln
            if spec is None:
                i = j
                continue
            kind, sub = spec[1], spec[3]
            if kind == "string":
                val = bytes(buf[i:j]).decode("utf-8", "replace")
            elif kind == "bytes":
                val = bytes(buf[i:j])
            elif kind == "msg":
                val = decode(buf, sub, i, j)
            else:  # packed repeated scalars
                vals = []
                k = i
                while k < j:
                    if kind == "varint":
                        v, k = _read_varint(buf, k)
                        vals.append(_signed(v))
                    elif kind == "float":
                        vals.append(struct.unpack_from("<f", buf, k)[0])
                        k += 4
                    else:
                        vals.append(struct.unpack_from("<d", buf, k)[0])
                        k += 8
                msg.setdefault(spec[0], []).extend(vals)
                i = j
                continue
            i = j
        else:
            raise ValueError(f"unsupported wire type {wt} in {name}")
        if spec is None:
            continue
        if spec[2]:
            msg[spec[0]].append(val)
        else:
            msg[spec[0]] = val
    return msg


# ------------------------------------------------------------------------------------------- .pdiparams streams
def write_lod_tensor(f, data_type, dims, raw):
    """One DenseTensor record: u32 version 0, u64 lod levels 0, u32 version 0, i32 desc size, TensorDesc, data."""
    f.write(struct.pack("<I", 0))
    f.write(struct.pack("<Q", 0))
    f.write(struct.pack("<I", 0))
    desc = encode({"data_type": data_type, "dims": [int(d) for d in dims]}, "TensorDesc")
    f.write(struct.pack("<i", len(desc)))
    f.write(desc)
    f.write(raw)


def read_lod_tensor(f):
    """-> (data_type, dims, raw bytes, lod) or None at EOF."""
    head = f.read(4)
    if len(head) < 4:
        return None
    (levels,) = struct.unpack("<Q", f.read(8))
    lod = []
    for _ in range(levels):
        (n,) = struct.unpack("<Q", f.read(8))
        lod.append(f.read(n))
    f.read(4)  # tensor version
    (dsz,) = struct.unpack("<i", f.read(4))
    desc = decode(f.read(dsz), "TensorDesc")
    dt, dims = desc.get("data_type", 5), desc.get("dims", [])
    n = 1
    for d in dims:
        n *= d
    raw = f.read(n * _ELT_BYTES[dt])
    return dt, dims, raw, lod


_ELT_BYTES = {0: 1, 1: 2, 2: 4, 3: 8, 4: 2, 5: 4, 6: 8, 20: 1, 21: 1, 22: 2, 23: 8, 24: 16}
