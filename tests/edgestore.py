"""Test helper: build Titan edgestore rows (what a scan hands to VertexJobConverter).

Uses the oracle's encoder (oracle/fulgora_ref.c, a restatement of EdgeSerializer.writeRelation,
EdgeSerializer.java:222-315) to write, for every vertex, one row holding:
  - the VertexExists system property entry (BaseKey.java:27-28; written for every vertex,
    StandardTitanTx.java:509),
  - optional Integer user properties,
  - one OUT entry per out-edge and one IN entry per in-edge (two entries per edge,
    StandardTitanGraph.java:564-591; a self-loop yields both on the same row),
sorted by column bytes (unsigned lexicographic, StaticArrayBuffer.java:381-393), in the
StaticArrayEntryList layout (StaticArrayEntryList.java:15-50).  Rows are ordered by
unsigned key, as an ordered scan returns them.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import fulgora as fr  # noqa: E402

PB = 5  # cluster.max-partitions = 32 (GraphDatabaseConfiguration.java:665)
VERTEX_EXISTS_ID = None


def user_edge_label(count):
    return fr.load().fr_schema_id(2, count)


def user_property_key(count):
    return fr.load().fr_schema_id(0, count)


def vertex_id(i, pb=PB):
    """Round-robin placement over 2^pb partitions (only the id layout matters)."""
    return fr.load().fr_vertex_id(i // (1 << pb) + 1, i % (1 << pb), pb)


def key_of(vid, pb=PB):
    return fr.load().fr_key_of(vid, pb)


@dataclass
class Rows:
    keys: np.ndarray
    entry_begin: np.ndarray
    byte_begin: np.ndarray
    data: np.ndarray
    limit_valpos: np.ndarray

    @property
    def nrows(self):
        return len(self.keys)

    def slice(self, a, b):
        """Rows [a, b) with their offsets rebased (a work block, or one rank's row range)."""
        eb, bb = self.entry_begin[a:b + 1], self.byte_begin[a:b + 1]
        return Rows(self.keys[a:b].copy(), (eb - eb[0]).copy(), (bb - bb[0]).copy(), self.data[bb[0]:bb[-1]].copy(),
                    self.limit_valpos[eb[0]:eb[-1]].copy())

    def save(self, path, **extra):
        np.savez_compressed(path, keys=self.keys, entry_begin=self.entry_begin, byte_begin=self.byte_begin,
                            data=self.data, limit_valpos=self.limit_valpos, **extra)

    @classmethod
    def load(cls, npz):
        return cls(npz["keys"], npz["entry_begin"], npz["byte_begin"], npz["data"], npz["limit_valpos"])


@dataclass
class GraphSpec:
    """Edges reference vertex indices; ids are assigned with vertex_id()."""
    n: int
    edges: list = field(default_factory=list)          # (src, dst, label_type_id, [(key, value)])
    vprops: dict = field(default_factory=dict)          # vertex -> [(key, value)]
    ghost_rows: list = field(default_factory=list)      # extra rows without VertexExists: (vid, edges as (dir, other_vid, label))
    schema_rows: int = 0                                # rows keyed by schema vertex ids (filtered)
    vids: list = None
    # vertex cuts (vertex labels made with partition(), TitanPartitionGraphTest.java:291-321):
    # their edges are stored on the representative in the other endpoint's partition
    partitioned: list = field(default_factory=list)
    pv_ghost: list = field(default_factory=list)       # partitioned vertices whose canonical row is absent


def partitioned_vertex_id(count, pb=PB):
    """Canonical id of a vertex cut (IDManager.getVertexID -> getCanonicalVertexIdFromCount, :500-528)."""
    lib = fr.load()
    return lib.fr_canonical_vertex_id(lib.fr_partitioned_vertex_id(count, 0, pb), pb)


def representative(pvid, partition, pb=PB):
    """IDManager.getPartitionedVertexId(pvid, partition) (:540-545)."""
    return fr.load().fr_partitioned_vertex_id(pvid >> (pb + 3), partition, pb)


def partition_of(vid, pb=PB):
    return (vid >> 3) & ((1 << pb) - 1)


def build_rows(spec: GraphSpec, schema: fr.OracleSchema, pb=PB, prop_types=None) -> tuple[Rows, np.ndarray]:
    prop_types = prop_types or {}
    vids = spec.vids if spec.vids is not None else [vertex_id(i, pb) for i in range(spec.n)]
    pset = set(spec.partitioned)
    vids = [partitioned_vertex_id(1000 + i, pb) if i in pset else v for i, v in enumerate(vids)]
    per_row = {v: [] for i, v in enumerate(vids) if i not in set(spec.pv_ghost)}
    rel = 1000
    for i, v in enumerate(vids):
        if i in set(spec.pv_ghost):
            continue
        rel += 1
        per_row[v].append(fr.encode_vertex_exists(rel))
        for key, val in spec.vprops.get(i, []):
            rel += 1
            per_row[v].append(fr.encode_property(key, prop_types.get(key, 3), val, rel))

    def placed(i, other_i):
        # a vertex cut keeps the edge on its representative in the other endpoint's partition
        return representative(vids[i], partition_of(vids[other_i], pb), pb) if i in pset else vids[i]

    for (s, d, label, props) in spec.edges:
        rel += 1
        vs, vd = placed(s, d), placed(d, s)
        per_row.setdefault(vs, []).append(fr.encode_edge(schema, label, 0, vd, rel, props))
        per_row.setdefault(vd, []).append(fr.encode_edge(schema, label, 1, vs, rel, props))
    for (gvid, gedges) in spec.ghost_rows:
        ents = []
        for (dr, other, label) in gedges:
            rel += 1
            ents.append(fr.encode_edge(schema, label, dr, other, rel, []))
        per_row[gvid] = ents
    for k in range(spec.schema_rows):
        sid = fr.load().fr_schema_id(0, 500 + k)   # a property-key schema vertex
        rel += 1
        per_row[sid] = [fr.encode_vertex_exists(rel)]
    keys = []
    for v in per_row:
        key = key_of(v, pb) if (v & 3) != 1 else v
        keys.append((key & ((1 << 64) - 1), v))
    keys.sort()
    data, lv, eb, bb, kk = bytearray(), [], [0], [0], []
    for ukey, v in keys:
        ents = sorted(per_row[v], key=lambda e: e[0][: e[1]])   # column = bytes before valuePos
        row_start = len(data)
        for b, vpos in ents:
            data += b
            lv.append(((len(data) - row_start) << 32) | vpos)
        eb.append(eb[-1] + len(ents))
        bb.append(len(data))
        kk.append(ukey - (1 << 64) if ukey >= (1 << 63) else ukey)
    rows = Rows(np.asarray(kk, np.int64), np.asarray(eb, np.int64), np.asarray(bb, np.int64),
                np.frombuffer(bytes(data), dtype=np.uint8).copy() if data else np.zeros(1, np.uint8),
                np.asarray(lv, np.int64))
    return rows, np.asarray(vids, np.int64)
