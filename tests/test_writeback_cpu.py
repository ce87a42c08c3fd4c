"""CPU: result write-back host logic — the compute-key column header against the
oracle's IDHandler restatement, the store merge (single-cardinality column overwrite, column
order, idempotence) and the property read-back, on oracle-encoded entries."""
import numpy as np
import pytest

import fulgora as fr
from titan_amd import _lib as L
from titan_amd.computer import _relation_type_header, merge_rows, read_property
from titan_amd.engine import Rows

lib = fr.load()


def uprop(count):
    return (count << 6) | 5


@pytest.mark.parametrize("count", [1, 2, 15, 16, 63, 64, 900, 5000, 1 << 20, (1 << 40) + 3])
def test_header_matches_oracle(count):
    # IDHandler.writeRelationType(keyId, PROPERTY_DIR, invisible=false) (IDHandler.java:88-94)
    assert _relation_type_header(uprop(count)) == fr.buf_bytes("fr_write_relation_type", uprop(count), 0, 0, 0)


def rows_of(per_row):
    """{vid: [(bytes, valuePos)]} -> Rows in unsigned key order, entries in column order."""
    keys = sorted(per_row, key=lambda v: lib.fr_key_of(v, 5) & ((1 << 64) - 1))
    data, lv, eb, bb, kk = bytearray(), [], [0], [0], []
    for v in keys:
        start = len(data)
        for b, vp in sorted(per_row[v], key=lambda e: e[0][:e[1]]):
            data += b
            lv.append(((len(data) - start) << 32) | vp)
        eb.append(len(lv))
        bb.append(len(data))
        kk.append(lib.fr_key_of(v, 5))
    return Rows(np.asarray(kk, np.int64), np.asarray(eb, np.int64), np.asarray(bb, np.int64),
                np.frombuffer(bytes(data), np.uint8).copy(), np.asarray(lv, np.int64))


def test_merge_overwrites_single_property_and_keeps_order():
    dist, pr = uprop(900), uprop(901)
    vids = [lib.fr_vertex_id(c, p, 5) for c, p in ((1, 0), (1, 3), (7, 31), (2, 9))]
    knows = lib.fr_schema_id(2, 1)
    s = fr.OracleSchema([{"type_id": knows, "multiplicity": 0}], [])
    store = rows_of({v: [fr.encode_vertex_exists(10 + i), fr.encode_edge(s, knows, 0, vids[(i + 1) % 4], 50 + i),
                         fr.encode_property(dist, L.DT_LONG, 99, 70 + i)] for i, v in enumerate(vids)})
    muts = rows_of({vids[0]: [fr.encode_property(dist, L.DT_LONG, 5, 1000)],
                    vids[2]: [fr.encode_property(dist, L.DT_LONG, -7, 1001), fr.encode_property_f64(pr, 0.25, 1002)]})
    merged = merge_rows(store, muts)
    assert list(merged.keys) == list(store.keys)                      # no new rows, same key order
    assert read_property(merged, vids[0], dist, L.DT_LONG) == 5       # overwritten
    assert read_property(merged, vids[1], dist, L.DT_LONG) == 99      # untouched
    assert read_property(merged, vids[2], dist, L.DT_LONG) == -7
    assert read_property(merged, vids[2], pr, L.DT_DOUBLE) == 0.25    # added
    assert read_property(merged, vids[3], pr, L.DT_DOUBLE) is None
    # entry count: + one new entry (pr on vids[2]); replacements keep the count
    assert merged.entry_begin[-1] == store.entry_begin[-1] + 1
    # idempotent, and every row still starts with VertexExists (column 0x02) so no ghost appears
    again = merge_rows(merged, muts)
    assert np.array_equal(again.data, merged.data) and np.array_equal(again.limit_valpos, merged.limit_valpos)
    for r in range(merged.nrows):
        assert merged.data[merged.byte_begin[r]] == 0x02


def test_merge_adds_rows_for_new_keys():
    dist = uprop(900)
    v0, v1 = lib.fr_vertex_id(3, 1, 5), lib.fr_vertex_id(4, 2, 5)
    store = rows_of({v0: [fr.encode_vertex_exists(1)]})
    merged = merge_rows(store, rows_of({v1: [fr.encode_property(dist, L.DT_LONG, 1, 2)]}))
    assert merged.nrows == 2
    assert read_property(merged, v1, dist, L.DT_LONG) == 1


def test_read_property_integer_values():
    deg = uprop(902)
    v = lib.fr_vertex_id(5, 0, 5)
    for val in (0, 1, -1, 2 ** 31 - 1, -2 ** 31):
        r = rows_of({v: [fr.encode_vertex_exists(1), fr.encode_property(deg, L.DT_INTEGER, val, 3)]})
        assert read_property(r, v, deg, L.DT_INTEGER) == val


def test_generic_key_known_answer():
    """A generic (Object) key's value: writeClassAndObject = VariableLong.writePositive of the
    class registration (Long 13, Double 20, Integer 12; StandardSerializer.java:71-81) and the
    serializer's bytes WITHOUT the null flag (:303-322) — hand-derived, then read back."""
    key = uprop(900)
    hdr = _relation_type_header(key)
    b, vp = fr.encode_property_generic(key, L.DT_LONG, 5, 3)
    assert vp == len(hdr) and b[:vp] == hdr
    assert b[vp:] == bytes([0x80 | 13]) + (5 + (1 << 63)).to_bytes(8, "big") + bytes([0x83])
    b, vp = fr.encode_property_generic(key, L.DT_INTEGER, -3, 3)
    assert b[vp:] == bytes([0x80 | 12, 0x80 | 7, 0x83])     # convert2Unsigned(-3) = |-3| << 1 | 1 = 7 (VariableLong.java:112-115)
    b, vp = fr.encode_property_generic(key, L.DT_DOUBLE, 0.5, 3)
    assert b[vp:] == bytes([0x80 | 20]) + bytes.fromhex("3fe0000000000000") + bytes([0x83])
    v = lib.fr_vertex_id(5, 0, 5)
    for dt, val in ((L.DT_LONG, -(1 << 40)), (L.DT_INTEGER, 2 ** 31 - 1), (L.DT_DOUBLE, 1.0 / 3)):
        r = rows_of({v: [fr.encode_vertex_exists(1), fr.encode_property_generic(key, dt, val, 7)]})
        assert read_property(r, v, key, L.DT_OBJECT) == val


def test_result_mode_defaults_follow_the_program():
    """An unset resultMode takes the program's getPreferredResultGraph / getPreferredPersist
    (FulgoraGraphComputer.java:133-135): PageRank / ShortestDistance persist into the original
    graph (PageRankVertexProgram.java:103-110, ShortestDistanceVertexProgram.java:81-88),
    DegreeCounter into a new one (OLAPTest.java:391-398); an explicit mode wins."""
    from titan_amd import DegreeCounter, GpuGraph, PageRankVertexProgram, ShortestDistanceVertexProgram
    from titan_amd.computer import TitanGraphComputer as TGC
    from titan_amd.generic import GenericVertexProgram
    g = GpuGraph(edges=(64, np.zeros(1, np.int32), np.ones(1, np.int32), None))
    for prog, mode in ((PageRankVertexProgram(), TGC.ResultMode.PERSIST),
                       (ShortestDistanceVertexProgram(8, 3), TGC.ResultMode.PERSIST),
                       (DegreeCounter(2), TGC.ResultMode.LOCALTX),
                       (GenericVertexProgram(), TGC.ResultMode.NONE)):
        c = g.compute().program(prog)
        assert c._result_mode() == (False, mode)
        c.resultMode(TGC.ResultMode.NONE)
        assert c._result_mode() == (True, TGC.ResultMode.NONE)
    assert g.compute()._result_mode() == (False, TGC.ResultMode.NONE)


def test_missing_compute_keys_become_generic_keys():
    """getOrCreatePropertyKey with the default schema maker: an unknown compute key is created
    generic (dataType(Object.class), DefaultSchemaMaker.java:46-48) with the next schema id."""
    from titan_amd import GpuGraph
    sd = {"edge_types": [{"type_id": lib.fr_schema_id(2, 7), "multiplicity": 0}], "property_keys": [[uprop(40), 3]]}
    g = GpuGraph(edges=(64, np.zeros(1, np.int32), np.ones(1, np.int32), None), schema=sd,
                 property_keys={"typed": (uprop(900), L.DT_LONG)})
    assert g.property_key("typed") == (uprop(900), L.DT_LONG)
    k1 = g.property_key("a")
    k2 = g.property_key("b")
    assert k1 == (uprop(901), L.DT_OBJECT) and k2 == (uprop(902), L.DT_OBJECT)
    assert g.property_key("a") == k1                                   # created once
