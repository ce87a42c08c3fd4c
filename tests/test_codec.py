"""CPU: edgestore codec known answers + the reference's round-trip properties.

Known answers are derived by hand from the Java sources (derivation in the comments);
round-trip properties restate VariableLongTest (ttest/graphdb/idmanagement/VariableLongTest.java:
100-155, 277-296) and IDManagementTest (:48-130).
"""
import ctypes as C
import random

import numpy as np
import pytest

import fulgora as fr

lib = fr.load()


def enc(fn, *a):
    return fr.buf_bytes(fn, *a)


def dec(fn, data: bytes, pos=0):
    arr = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data if data else b"\0")
    p = C.c_size_t(pos)
    v = getattr(lib, fn)(C.cast(arr, C.POINTER(C.c_uint8)), C.byref(p))
    return v, p.value


# ---------------------------------------------------------------- hand-derived vectors
def test_positive_varint_vectors():
    # writeUnsigned: 7-bit groups MSB first, stop bit 0x80 on the LAST byte (VariableLong.java:46-57)
    assert enc("fr_vl_write_positive", 0) == b"\x80"
    assert enc("fr_vl_write_positive", 127) == b"\xff"
    assert enc("fr_vl_write_positive", 128) == b"\x01\x80"
    assert enc("fr_vl_write_positive", 300) == b"\x02\xac"      # 300 = 2*128 + 44


def test_zigzag_vectors():
    # convert2Unsigned: |v|<<1 | sign (VariableLong.java:112-115)
    assert enc("fr_vl_write", 1) == b"\x82"
    assert enc("fr_vl_write", -1) == b"\x83"
    assert enc("fr_vl_write", 0) == b"\x80"


def test_backward_vectors():
    # writeUnsignedBackward: >= 3 bytes, first byte = 0x80 | (nbytes-3)<<4 | top 4 bits (:234-252)
    assert enc("fr_vl_write_positive_backward", 0) == b"\x80\x00\x00"
    assert enc("fr_vl_write_positive_backward", 5) == b"\x80\x00\x05"
    assert enc("fr_vl_write_positive_backward", 1 << 20) == b"\x90\x40\x00\x00"


def test_relation_type_vectors():
    # user edge label count c has id c<<6 | 21 (IDManager UserEdgeLabel); column prefix
    # 0b011 (user, edge) + prefixed varint (c<<1 | dir) (IDHandler.java:88-94)
    lab1 = lib.fr_schema_id(2, 1)
    assert lab1 == (1 << 6) | 21
    assert enc("fr_write_relation_type", lab1, 1, 0, 0) == b"\x62"   # OUT
    assert enc("fr_write_relation_type", lab1, 1, 1, 0) == b"\x63"   # IN
    lab8 = lib.fr_schema_id(2, 8)
    assert enc("fr_write_relation_type", lab8, 1, 0, 0) == b"\x70\x90"   # continue mask + 1 byte
    # VertexExists: system property key count 1 -> prefix 0, value 2 -> single byte 0x02
    assert enc("fr_write_relation_type", lib.fr_schema_id(1, 1), 0, 0, 1) == b"\x02"
    b, vpos = fr.encode_vertex_exists(7)
    assert b[0] == 0x02 and vpos == 1 and b[1] == 0x00       # null flag then Boolean


def test_vertex_key_vectors():
    # pb=5, count=1, partition=3: id = ((1<<5)+3)<<3 = 280; key = 3<<59 | 1<<3 (IDManager :461-473)
    vid = lib.fr_vertex_id(1, 3, 5)
    assert vid == 280
    assert lib.fr_key_of(vid, 5) & ((1 << 64) - 1) == (3 << 59) | 8
    assert lib.fr_key_id(lib.fr_key_of(vid, 5), 5) == vid


# ---------------------------------------------------------------- round-trip properties
def test_varint_roundtrip_random():
    rnd = random.Random(1)
    for _ in range(2000):
        v = rnd.getrandbits(rnd.randrange(1, 63))
        b = enc("fr_vl_write_positive", v)
        assert len(b) == lib.fr_vl_positive_length(v)
        assert dec("fr_vl_read_positive", b) == (v, len(b))
        s = v if rnd.random() < 0.5 else -v
        assert dec("fr_vl_read", enc("fr_vl_write", s))[0] == s
        bb = enc("fr_vl_write_positive_backward", v)
        assert len(bb) == lib.fr_vl_backward_length(v)
        val, start = dec("fr_vl_read_positive_backward", bb, len(bb))
        assert (val, start) == (v, 0)


def test_prefix_roundtrip():
    rnd = random.Random(2)
    for _ in range(2000):
        v = rnd.getrandbits(rnd.randrange(1, 60))
        prefix = rnd.randrange(8)
        b = enc("fr_vl_write_positive_with_prefix", v, prefix, 3)
        arr = (C.c_uint8 * len(b)).from_buffer_copy(b)
        p = C.c_size_t(0)
        val, pre = C.c_int64(), C.c_int64()
        lib.fr_vl_read_positive_with_prefix(C.cast(arr, C.POINTER(C.c_uint8)), C.byref(p), 3, C.byref(val), C.byref(pre))
        assert (val.value, pre.value, p.value) == (v, prefix, len(b))


def test_backward_encoding_is_byte_order_preserving():
    # VariableLongTest :277-296 — this is what sorts MULTI-edge columns by other vertex id
    rnd = random.Random(3)
    vals = sorted({rnd.getrandbits(rnd.randrange(1, 50)) for _ in range(3000)})
    encs = [enc("fr_vl_write_positive_backward", v) for v in vals]
    assert encs == sorted(encs)


def test_key_roundtrip_random():
    rnd = random.Random(4)
    for pb in (0, 1, 5, 8, 16):
        for _ in range(500):
            count = rnd.randrange(1, 1 << (60 - 3 - pb))
            part = rnd.randrange(1 << pb) if pb else 0
            vid = lib.fr_vertex_id(count, part, pb)
            assert lib.fr_key_id(lib.fr_key_of(vid, pb), pb) == vid


@pytest.mark.parametrize("mult", [0, 1, 2, 3, 4])
def test_edge_entry_roundtrip(mult):
    lab = lib.fr_schema_id(2, 3)
    w = lib.fr_schema_id(0, 1)
    other_key = lib.fr_schema_id(0, 2)
    s = fr.OracleSchema([{"type_id": lab, "multiplicity": mult, "signature": [w]}], [(w, 3), (other_key, 4)])
    rnd = random.Random(mult)
    for _ in range(200):
        other = lib.fr_vertex_id(rnd.randrange(1, 1 << 30), rnd.randrange(32), 5)
        rid = rnd.randrange(1, 1 << 40)
        wt = rnd.randrange(-(1 << 31), 1 << 31)
        d = rnd.randrange(2)
        props = [(w, wt), (other_key, rnd.randrange(-(1 << 62), 1 << 62))]
        b, vpos = fr.encode_edge(s, lab, d, other, rid, props)
        arr = (C.c_uint8 * len(b)).from_buffer_copy(b)
        out = [C.c_int64(), C.c_int(), C.c_int64(), C.c_int64(), C.c_int(), C.c_int64()]
        rc = lib.fr_decode_edge(C.cast(arr, C.POINTER(C.c_uint8)), len(b), vpos, C.byref(s.s), w,
                                C.byref(out[0]), C.byref(out[1]), C.byref(out[2]), C.byref(out[3]),
                                C.byref(out[4]), C.byref(out[5]))
        assert rc == 0
        assert (out[0].value, out[1].value, out[2].value, out[3].value, out[4].value, out[5].value) == \
            (lab, d, other, rid, 1, wt)
