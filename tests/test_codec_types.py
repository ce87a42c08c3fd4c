"""CPU: the codec's datatype breadth — every attribute serializer in its normal
and byte-ordered (sort-key) form, the DESC sort-order byte flip, and weights stored in a MULTI
label's sort key — first as known answers for the oracle, then the product decoder
(tgo_decode_edge_entry, the host half of tgo_load_rows) against the oracle on random entries.

Known answers are derived by hand from the Java serializers (derivations in the comments;
paths under titan-core/.../graphdb/database/serialize/attribute/ unless noted).
"""
import ctypes as C
import random

import numpy as np
import pytest

import fulgora as fr
from titan_amd import _lib as L
from titan_amd.engine import Schema

lib = fr.load()
BYTE, SHORT, INTEGER, LONG, FLOAT, DOUBLE, BOOLEAN, DATE, CHARACTER, STRING = range(1, 11)
ALL_TYPES = [BYTE, SHORT, INTEGER, LONG, FLOAT, DOUBLE, BOOLEAN, DATE, CHARACTER, STRING]


def val(dt, value, byte_order=False, present=True):
    return fr.buf_bytes("fr_write_value", dt, 1 if present else 0, value, 1 if byte_order else 0)


# ---------------------------------------------------------------- known answers
def test_integer_and_long_forms():
    # normal Integer: null flag 0 + zig-zag varint (IntegerSerializer.java:20-23; VariableLong.java:125-127)
    assert val(INTEGER, 5) == b"\x00\x8a"
    # byte order: putInt(v - Integer.MIN_VALUE) (IntegerSerializer.java:31-33) = v ^ 0x80000000, big-endian
    assert val(INTEGER, 5, True) == b"\x00\x80\x00\x00\x05"
    assert val(INTEGER, -1, True) == b"\x00\x7f\xff\xff\xff"
    # Long / Date: putLong(v - Long.MIN_VALUE) in both forms (LongSerializer.java:20-32; DateSerializer)
    assert val(LONG, 1) == b"\x00\x80\x00\x00\x00\x00\x00\x00\x01"
    assert val(DATE, 0, True) == b"\x00\x80" + b"\x00" * 7
    # null: flag byte -1 (StandardSerializer.java:286-301)
    assert val(INTEGER, 0, present=False) == b"\xff"


def test_float_double_forms():
    # normal: raw IEEE bits (FloatSerializer.java:33-36 putFloat)
    assert val(FLOAT, 1) == b"\x00\x3f\x80\x00\x00"
    assert val(DOUBLE, 2) == b"\x00\x40" + b"\x00" * 7
    # byte order: floatToSortableInt (bits ^ (bits>>31 & 0x7fffffff), NumericUtils.java:58-79)
    # then IntegerSerializer.writeByteOrder (^ 0x80000000): 1.0f 0x3f800000 -> 0xbf800000
    assert val(FLOAT, 1, True) == b"\x00\xbf\x80\x00\x00"
    # -1.0f = 0xbf800000 -> ^0x7fffffff = 0xc07fffff -> ^0x80000000 = 0x407fffff
    assert val(FLOAT, -1, True) == b"\x00\x40\x7f\xff\xff"
    assert val(DOUBLE, 2, True) == b"\x00\xc0" + b"\x00" * 7


def test_character_byte_boolean_forms():
    # Character: ShortSerializer of (c + Short.MIN_VALUE) -> putShort(c) (CharacterSerializer.java)
    assert val(CHARACTER, ord("A")) == b"\x00\x00\x41"
    assert val(BYTE, -128) == b"\x00\x00"          # ByteSerializer: b - Byte.MIN_VALUE
    assert val(SHORT, 1) == b"\x00\x80\x01"
    assert val(BOOLEAN, 1) == b"\x00\x01"


def test_string_forms():
    # StringSerializer handles null itself (SupportsNullSerializer: no flag byte).
    # "" : writePositive(1 << 4) = 16 -> 0x90 (StringSerializer.java:153)
    assert val(STRING, 0) == b"\x90"
    # "12": ASCII marker 2 << 4 = 32 -> 0xa0, then chars, the last one | 0x80
    assert val(STRING, 12) == b"\xa0\x31\xb2"
    # value -5 -> U+00E9 U+2135 '5': full UTF, (3 << 4) + (1 << 3) = 56 -> 0xb8;
    # U+00E9 -> c3 a9, U+2135 -> e2 84 b5 (StringSerializer.java:160-176)
    assert val(STRING, -5) == b"\xb8\xc3\xa9\xe2\x84\xb5\x35"
    assert val(STRING, 0, present=False) == b"\x80"
    # byte order: 0 prefix, 2-byte chars, (char) 0 terminator (StringSerializer.java:54-67)
    assert val(STRING, 12, True) == b"\x00\x00\x31\x00\x32\x00\x00"
    assert val(STRING, 0, True, present=False) == b"\xff"


KNOWS = lib.fr_schema_id(2, 3)
W = lib.fr_schema_id(0, 1)        # Integer weight
K = {dt: lib.fr_schema_id(0, 10 + dt) for dt in ALL_TYPES}   # one property key per datatype
PKEYS = [(W, INTEGER)] + [(K[dt], dt) for dt in ALL_TYPES]


def schema_dict(mult=0, sort_key=(), signature=(), order="ASC"):
    return {"edge_types": [{"type_id": KNOWS, "multiplicity": mult, "sort_key": list(sort_key),
                            "signature": list(signature), "order": order}],
            "property_keys": [list(p) for p in PKEYS]}


def osch(sd):
    return fr.OracleSchema(sd["edge_types"], [tuple(p) for p in sd["property_keys"]])


def test_desc_sort_key_bytes_are_inverted():
    # EdgeSerializer.java:311-313: the sort-key bytes [keyStart, keyEnd) are flipped (~b)
    for order in ("ASC", "DESC"):
        s = osch(schema_dict(sort_key=[W], order=order))
        b, vp = fr.encode_edge(s, KNOWS, 0, 8, 1, [(W, 5)])
        key = b[1:6]            # after the one-byte relation type
        want = b"\x00\x80\x00\x00\x05"
        assert key == (want if order == "ASC" else bytes(x ^ 0xFF for x in want))


@pytest.mark.parametrize("order", ["ASC", "DESC"])
def test_sort_key_orders_columns(order):
    # entries of one label/direction sort by their sort key in column byte order: ascending
    # weights for ASC, descending for DESC (the flip makes byte order reverse value order)
    s = osch(schema_dict(sort_key=[W], order=order))
    rnd = random.Random(5)
    ws = [rnd.randrange(-1000, 1000) for _ in range(200)]
    ents = [fr.encode_edge(s, KNOWS, 0, 8 + 8 * i, 100 + i, [(W, w)]) for i, w in enumerate(ws)]
    by_col = [ws[i] for i in sorted(range(len(ws)), key=lambda i: ents[i][0][: ents[i][1]])]
    assert by_col == sorted(ws, reverse=(order == "DESC"))


def _oracle_decode(s, b, vp, weight_key):
    arr = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    out = [C.c_int64(), C.c_int(), C.c_int64(), C.c_int64(), C.c_int(), C.c_int64()]
    rc = lib.fr_decode_edge(C.cast(arr, C.POINTER(C.c_uint8)), len(b), vp, C.byref(s.s), weight_key,
                            *[C.byref(o) for o in out])
    return rc, [o.value for o in out]


def _product_decode(sd, b, vp, weight_key, labels=()):
    sch = Schema.from_dict(sd)
    lab = np.asarray(labels, np.int64)
    opts = L.LoadOpts(scope=0, apply_cap=1, n_labels=len(lab), label_ids=L.ptr(lab, C.c_int64) if len(lab) else None,
                      weight_key=weight_key)
    arr = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    e = L.EdgeEntry()
    rc = L.load().tgo_decode_edge_entry(C.byref(sch.c), C.byref(opts), C.cast(arr, C.POINTER(C.c_uint8)),
                                        len(b), vp, C.byref(e))
    return rc, e


def random_props(rnd, keys):
    out = []
    for k in keys:
        dt = dict(PKEYS)[k]
        if rnd.random() < 0.1:
            continue                                 # property absent (null inline / not written)
        if dt in (STRING,):
            v = rnd.choice([0, rnd.randrange(1, 10 ** 9), -rnd.randrange(1, 10 ** 6)])
        elif dt == CHARACTER:
            v = rnd.randrange(1, 0xFFFF)
        elif dt in (BYTE,):
            v = rnd.randrange(-128, 128)
        elif dt == SHORT:
            v = rnd.randrange(-32768, 32768)
        elif dt == BOOLEAN:
            v = rnd.randrange(2)
        elif dt in (INTEGER,):
            v = rnd.randrange(-(1 << 31), 1 << 31)
        else:
            v = rnd.randrange(-(1 << 50), 1 << 50)
        out.append((k, v))
    return out


LAYOUTS = [
    # (multiplicity, sort key, signature, order): where the weight sits and what precedes it
    (0, [K[STRING], K[FLOAT], K[DATE], W], [], "ASC"),
    (0, [K[STRING], K[FLOAT], K[DATE], W], [], "DESC"),
    (0, [K[CHARACTER], K[DOUBLE], K[LONG], K[BYTE], K[SHORT], K[BOOLEAN], W], [], "DESC"),
    (0, [W, K[STRING]], [K[STRING], K[DOUBLE]], "DESC"),
    (0, [K[STRING]], [K[STRING], K[FLOAT], W], "ASC"),
    (0, [K[DATE]], [], "DESC"),                                  # weight among remaining properties
    (1, [], [K[STRING], W], "ASC"),                              # SIMPLE: value-side signature
    (3, [], [], "ASC"),                                          # ONE2MANY: remaining only
]


@pytest.mark.parametrize("layout", range(len(LAYOUTS)))
def test_product_decoder_matches_oracle(layout):
    mult, sk, sig, order = LAYOUTS[layout]
    sd = schema_dict(mult, sk, sig, order)
    s = osch(sd)
    rnd = random.Random(100 + layout)
    all_keys = [W] + [K[dt] for dt in ALL_TYPES]
    for _ in range(300):
        other = lib.fr_vertex_id(rnd.randrange(1, 1 << 30), rnd.randrange(32), 5)
        rid = rnd.randrange(1, 1 << 40)
        d = rnd.randrange(2)
        props = random_props(rnd, all_keys)
        b, vp = fr.encode_edge(s, KNOWS, d, other, rid, props)
        orc, o = _oracle_decode(s, b, vp, W)
        prc, e = _product_decode(sd, b, vp, W)
        assert orc == 0 and prc == 0
        assert (e.type_id, e.dir, e.other_id) == (o[0], o[1], o[2]) == (KNOWS, d, other)
        assert (e.has_weight, e.weight if e.has_weight else 0) == (o[4], o[5] if o[4] else 0)
        assert e.has_weight == (W in dict(props))
        if e.has_weight:
            assert e.weight == dict(props)[W]
        # no weight requested: the topology alone
        prc, e0 = _product_decode(sd, b, vp, 0)
        assert prc == 0 and (e0.other_id, e0.has_weight) == (other, 0)


@pytest.mark.parametrize("dt", [DATE, STRING])
def test_unsupported_weight_key_is_rejected(dt):
    # Date and String weights have no edge function here (and ShortestDistanceVertexProgram.java:53
    # casts edge.<Integer>value: a ClassCastException in the reference)
    sd = schema_dict(0, [K[dt]], [])
    s = osch(sd)
    b, vp = fr.encode_edge(s, KNOWS, 0, 8, 1, [(K[dt], 3)])
    E_UNSUPPORTED = -7                     # TGO_E_UNSUPPORTED / FR_E_UNSUPPORTED
    assert _oracle_decode(s, b, vp, K[dt])[0] == E_UNSUPPORTED
    assert _product_decode(sd, b, vp, K[dt])[0] == E_UNSUPPORTED


@pytest.mark.parametrize("dt", [LONG, DOUBLE])
@pytest.mark.parametrize("where", ["sort_key", "signature", "remaining"])
def test_wide_weight_keys_decode_to_64_bits(dt, where):
    """Long and Double weight keys (generic edge functions): the oracle reads
    the 64-bit value — the Long, or the Double's IEEE bits (DoubleSerializer.java:25-41: putDouble,
    byte order doubleToSortableLong then the Long flip) — in every position and sort order; the
    product's single-entry call rejects them (its weight field is 32 bits), the row loads carry
    them in a value table (tests/test_gpu_generic.py)."""
    import struct
    vals = [-(1 << 40) - 3, -1, 0, 7, 5_000_000_000] if dt == LONG else [-1099511627779, -2, 0, 3, 1 << 53]
    for order in ("ASC", "DESC"):
        sd = schema_dict(0, [K[dt]] if where == "sort_key" else [], [K[dt]] if where == "signature" else [], order)
        s = osch(sd)
        for i, x in enumerate(vals):
            b, vp = fr.encode_edge(s, KNOWS, i % 2, 8 + 8 * i, 100 + i, [(K[dt], x)])
            orc, o = _oracle_decode(s, b, vp, K[dt])
            assert orc == 0 and o[4] == 1
            want = x if dt == LONG else struct.unpack("<q", struct.pack("<d", float(x)))[0]
            assert o[5] == want, (dt, where, order, x)
            assert _product_decode(sd, b, vp, K[dt])[0] == -7


@pytest.mark.parametrize("dt", [BYTE, SHORT, CHARACTER, BOOLEAN, FLOAT])
@pytest.mark.parametrize("where", ["sort_key", "signature", "remaining"])
def test_32_bit_weight_datatypes_decode_alike(dt, where):
    """A weight of any datatype that fits 32 bits (generic programs' edge functions read it):
    integral values as integers, a Float as its IEEE bits (-0.0 as +0.0), in the sort key (ASC /
    DESC byte-ordered form), the signature or the remaining properties; oracle == product."""
    import struct
    vals = {BYTE: [-128, -1, 0, 5, 127], SHORT: [-32768, -3, 0, 7, 32767], CHARACTER: [0, 65, 65535],
            BOOLEAN: [0, 1], FLOAT: [-7, -1, 0, 3, 1000]}[dt]
    for order in ("ASC", "DESC"):
        sd = schema_dict(0, [K[dt]] if where == "sort_key" else [], [K[dt]] if where == "signature" else [], order)
        s = osch(sd)
        for i, x in enumerate(vals):
            b, vp = fr.encode_edge(s, KNOWS, i % 2, 8 + 8 * i, 100 + i, [(K[dt], x)])
            orc, o = _oracle_decode(s, b, vp, K[dt])
            prc, e = _product_decode(sd, b, vp, K[dt])
            assert orc == 0 and prc == 0 and e.has_weight == 1 == o[4]
            want = struct.unpack("<i", struct.pack("<f", float(x)))[0] if dt == FLOAT else x
            if dt == FLOAT and x == 0:
                want = 0
            assert e.weight == o[5] == want, (dt, where, order, x)


def test_compressed_string_is_skipped():
    # a GZIP string (> 16000 chars) is (len << 3) + compressor id, then len raw bytes
    # (StringSerializer.java:177-184); a decoder that only skips it must land after it
    sd = {"edge_types": [{"type_id": KNOWS, "multiplicity": 1, "signature": [K[STRING], W]}],
          "property_keys": [list(p) for p in PKEYS]}
    s = osch(sd)
    b, vp = fr.encode_edge(s, KNOWS, 0, 8, 1, [(K[STRING], 7), (W, 42)])
    plain = val(STRING, 7)
    i = b.index(plain, vp)
    payload = bytes(range(37))
    gz = fr.buf_bytes("fr_vl_write_positive", (len(payload) << 3) + 1) + payload
    b2 = b[:i] + gz + b[i + len(plain):]
    rc, o = _oracle_decode(s, b2, vp, W)
    assert rc == 0 and (o[4], o[5]) == (1, 42)
    prc, e = _product_decode(sd, b2, vp, W)
    assert prc == 0 and (e.has_weight, e.weight) == (1, 42)


def test_typed_scope_skips_other_labels():
    other_label = lib.fr_schema_id(2, 4)
    sd = {"edge_types": [{"type_id": KNOWS, "multiplicity": 0}, {"type_id": other_label, "multiplicity": 0}],
          "property_keys": [list(p) for p in PKEYS]}
    s = osch(sd)
    b, vp = fr.encode_edge(s, other_label, 1, 16, 3, [])
    rc, e = _product_decode(sd, b, vp, 0, labels=[KNOWS])
    assert rc == 0 and e.selected == 0
    rc, e = _product_decode(sd, b, vp, 0, labels=[other_label])
    assert rc == 0 and e.selected == 1 and e.other_id == 16


def test_malformed_entries_fail():
    sd = schema_dict(0, [W], [], "DESC")
    s = osch(sd)
    b, vp = fr.encode_edge(s, KNOWS, 0, 8, 1, [(W, 5)])
    for cut in (1, 3):                                   # truncated inside the sort key
        rc, _ = _product_decode(sd, b[:cut], min(vp, cut), W)
        assert rc != 0
