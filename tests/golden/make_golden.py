"""Generate the golden fixtures under tests/golden/ (committed; re-run to regenerate).

Every fixture is edgestore rows (built with the restated encoder, tests/edgestore.py) plus
expected outputs taken from the REFERENCE'S OWN known answers — not from the oracle:

  gotg.npz            GraphOfTheGodsFactory.java:92-127 (12 vertices, 17 edges); expected
                      BFS levels / DegreeCounter values are the SURVEY.md §8c hand-derived
                      anchors, recomputed here by a plain BFS over the edge list.
  pagerank_tree.npz   OLAPTest.testPageRank (:476-519): complete 6-ary tree of depth 5,
                      child->parent `likes`, N = 9331, alpha = 0.85, iterations(10); the
                      closed form correctPR[d] = (1-a)/N + a*6*correctPR[d+1].
  sssp_tree.npz       OLAPTest.testShortestDistance (:564-621): random tree grown around the
                      seed, `connect` edges child->parent with signature(distance) weights
                      1..3; expected distance = the generated `distance` property.
  degree_random.npz   OLAPTest.generateRandomGraph (:61-88): vertex i has i+1 `knows`
                      out-edges; DegreeCounter(1) => degree == uid (:193-220) and
                      DegreeCounter(2) => sum of out-neighbour out-degrees (:241-279).

java.util.Random is unseeded in the reference (OLAPTest.java:39); here the generators are
seeded so the fixtures are reproducible.  The String-typed GotG properties (`name`,
`reason`) and the Geoshape `place` are not written (signature slots of absent properties are
serialized as the null flag 0xFF, StandardSerializer.java:292-296); nothing on the traversal
path reads them.
"""
from __future__ import annotations

import json
import os
import random
import sys
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import edgestore as es  # noqa: E402
import fulgora as fr  # noqa: E402

MULTI, SIMPLE, MANY2ONE, ONE2MANY, ONE2ONE = 0, 1, 2, 3, 4
DT_INTEGER = 3


def schema_dict(edge_types, property_keys):
    return {"edge_types": edge_types, "property_keys": property_keys}


def oracle_schema(sd):
    return fr.OracleSchema(sd["edge_types"], [tuple(x) for x in sd["property_keys"]])


def save(name, rows, vids, sd, **expected):
    rows.save(os.path.join(HERE, name + ".npz"), vids=vids, **{k: np.asarray(v) for k, v in expected.items()})
    with open(os.path.join(HERE, name + ".schema.json"), "w") as f:
        json.dump(sd, f, indent=1, sort_keys=True)


def bfs_levels(n, adj_lists, seed):
    lvl = [-1] * n
    lvl[seed] = 0
    dq = deque([seed])
    while dq:
        u = dq.popleft()
        for v in adj_lists[u]:
            if lvl[v] < 0:
                lvl[v] = lvl[u] + 1
                dq.append(v)
    return lvl


def make_gotg():
    L = {name: es.user_edge_label(i + 1) for i, name in enumerate(["father", "mother", "battled", "lives", "pet", "brother"])}
    time_key = es.user_property_key(1)
    reason_key = es.user_property_key(2)   # String: not encodable here, always null
    age_key = es.user_property_key(3)
    sd = schema_dict(
        [{"type_id": L["father"], "multiplicity": MANY2ONE},
         {"type_id": L["mother"], "multiplicity": MANY2ONE},
         {"type_id": L["battled"], "multiplicity": MULTI, "signature": [time_key]},
         {"type_id": L["lives"], "multiplicity": MULTI, "signature": [reason_key]},
         {"type_id": L["pet"], "multiplicity": MULTI},
         {"type_id": L["brother"], "multiplicity": MULTI}],
        [[time_key, DT_INTEGER], [age_key, DT_INTEGER]])
    names = ["saturn", "sky", "sea", "jupiter", "neptune", "hercules", "alcmene", "pluto",
             "nemean", "hydra", "cerberus", "tartarus"]
    ix = {n: i for i, n in enumerate(names)}
    ages = {"saturn": 10000, "jupiter": 5000, "neptune": 4500, "hercules": 30, "alcmene": 45, "pluto": 4000}
    E = [("jupiter", "saturn", "father", []), ("jupiter", "sky", "lives", []),
         ("jupiter", "neptune", "brother", []), ("jupiter", "pluto", "brother", []),
         ("neptune", "sea", "lives", []), ("neptune", "jupiter", "brother", []),
         ("neptune", "pluto", "brother", []), ("hercules", "jupiter", "father", []),
         ("hercules", "alcmene", "mother", []), ("hercules", "nemean", "battled", [(time_key, 1)]),
         ("hercules", "hydra", "battled", [(time_key, 2)]), ("hercules", "cerberus", "battled", [(time_key, 12)]),
         ("pluto", "jupiter", "brother", []), ("pluto", "neptune", "brother", []),
         ("pluto", "tartarus", "lives", []), ("pluto", "cerberus", "pet", []),
         ("cerberus", "tartarus", "lives", [])]
    assert len(E) == 17
    spec = es.GraphSpec(n=12, edges=[(ix[a], ix[b], L[l], p) for a, b, l, p in E],
                        vprops={ix[k]: [(age_key, v)] for k, v in ages.items()})
    # one ghost row (entries of a removed vertex, no VertexExists — OLAPTest.removeGhostVertices)
    ghost_vid = es.vertex_id(40)
    spec.vids = [es.vertex_id(i) for i in range(12)]
    spec.ghost_rows = [(ghost_vid, [(0, spec.vids[ix["jupiter"]], L["brother"])])]
    spec.schema_rows = 1
    rows, vids = es.build_rows(spec, oracle_schema(sd), prop_types={age_key: DT_INTEGER})
    out_l = [[] for _ in range(12)]
    in_l = [[] for _ in range(12)]
    for a, b, _, _ in E:
        out_l[ix[a]].append(ix[b])
        in_l[ix[b]].append(ix[a])
    both = [out_l[i] + in_l[i] for i in range(12)]
    INF = -1
    exp = {
        # inE: a receiver walks its OUT edges, so the distance spreads from w to every v
        # with v->w (against the edge); outE spreads along the edge.
        "bfs_in_saturn": bfs_levels(12, in_l, ix["saturn"]),
        "bfs_out_jupiter": bfs_levels(12, out_l, ix["jupiter"]),
        "bfs_both_jupiter": bfs_levels(12, both, ix["jupiter"]),
        "degree1": [len(out_l[i]) for i in range(12)],
    }
    # SURVEY.md §8c anchors (hand-derived from the GotG edge list)
    a = exp["bfs_in_saturn"]
    assert a[ix["saturn"]] == 0 and a[ix["jupiter"]] == 1
    assert all(a[ix[k]] == 2 for k in ["neptune", "hercules", "pluto"]) and sum(x == INF for x in a) == 7
    b = exp["bfs_out_jupiter"]
    assert [b[ix[k]] for k in ["saturn", "sky", "neptune", "pluto"]] == [1] * 4
    assert [b[ix[k]] for k in ["sea", "tartarus", "cerberus"]] == [2] * 3
    assert all(b[ix[k]] == INF for k in ["hercules", "alcmene", "nemean", "hydra"])
    c = exp["bfs_both_jupiter"]
    assert [c.count(0), c.count(1), c.count(2)] == [1, 5, 6]
    d = exp["degree1"]
    assert (d[ix["jupiter"]], d[ix["neptune"]], d[ix["hercules"]], d[ix["pluto"]], d[ix["cerberus"]]) == (4, 3, 5, 4, 1)
    assert sum(d) == 17
    save("gotg", rows, vids, sd, names=np.array(names), **{k: np.asarray(v, np.int64) for k, v in exp.items()},
         ghost_vid=np.int64(ghost_vid))


def make_pagerank_tree():
    likes, knows = es.user_edge_label(1), es.user_edge_label(2)
    sd = schema_dict([{"type_id": likes, "multiplicity": MULTI}, {"type_id": knows, "multiplicity": MULTI}], [])
    branch, diameter, alpha = 6, 5, 0.85
    numV = (branch ** (diameter + 1) - 1) // (branch - 1)
    assert numV == 9331
    depth = [0]
    edges = []

    def expand(v, d):        # OLAPTest.expand :476-493 (recursive, children then grandchildren)
        if d < diameter:
            for _ in range(branch):
                u = len(depth)
                depth.append(d + 1)
                edges.append((u, v, likes, []))
                expand(u, d + 1)
    expand(0, 0)
    assert len(depth) == numV
    correct = [0.0] * (diameter + 1)
    for i in range(diameter, -1, -1):
        pr = (1.0 - alpha) / numV
        if i < diameter:
            pr += alpha * branch * correct[i + 1]
        correct[i] = pr
    spec = es.GraphSpec(n=numV, edges=edges)
    rows, vids = es.build_rows(spec, oracle_schema(sd))
    save("pagerank_tree", rows, vids, sd, depth=np.asarray(depth, np.int64),
         expected_pr=np.asarray([correct[d] for d in depth]), alpha=np.float64(alpha),
         iterations=np.int64(10), num_v=np.int64(numV))


def make_sssp_tree(seed=20251015):
    dist_key = es.user_property_key(1)
    connect = es.user_edge_label(1)
    sd = schema_dict([{"type_id": connect, "multiplicity": MULTI, "signature": [dist_key]}], [[dist_key, DT_INTEGER]])
    rnd = random.Random(seed)
    max_depth, max_branch = 16, 5
    dist = [0]
    edges = []

    def grow(v, depth):      # OLAPTest.growVertex :609-621 (loop bound re-drawn every test)
        if depth >= max_depth:
            return
        i = 0
        while i < rnd.randrange(max_branch) + 1:
            w = rnd.randrange(3) + 1
            n = len(dist)
            dist.append(depth + w)
            edges.append((n, v, connect, [(dist_key, w)]))
            grow(n, depth + w)
            i += 1
    grow(0, 0)
    spec = es.GraphSpec(n=len(dist), edges=edges)
    rows, vids = es.build_rows(spec, oracle_schema(sd))
    save("sssp_tree", rows, vids, sd, expected_dist=np.asarray(dist, np.int64), seed_index=np.int64(0),
         max_depth=np.int64(max_depth + 4), weight_key=np.int64(dist_key))


def make_degree_random(num_v, name, seed):
    uid_key = es.user_property_key(1)
    knows = es.user_edge_label(1)
    sd = schema_dict([{"type_id": knows, "multiplicity": MULTI}], [[uid_key, DT_INTEGER]])
    rnd = random.Random(seed)
    edges = []
    out = [[] for _ in range(num_v)]
    for i in range(num_v):
        for _ in range(i + 1):
            u = rnd.randrange(num_v)
            edges.append((i, u, knows, []))
            out[i].append(u)
    assert num_v * (num_v + 1) == 2 * len(edges)
    spec = es.GraphSpec(n=num_v, edges=edges, vprops={i: [(uid_key, i + 1)] for i in range(num_v)})
    rows, vids = es.build_rows(spec, oracle_schema(sd), prop_types={uid_key: DT_INTEGER})
    degree1 = [i + 1 for i in range(num_v)]
    degree2 = [sum(len(out[w]) for w in out[v]) for v in range(num_v)]
    save(name, rows, vids, sd, degree1=np.asarray(degree1, np.int64), degree2=np.asarray(degree2, np.int64))


def make_partition_groups(group_degrees=(10, 20, 30), ghost_degree=5):
    """TitanPartitionGraphTest.setupGroupClusters (:291-321): each group vertex has a
    partition() label (a vertex cut); person k of group i has member person->group and
    contain group->person.  testVertexPartitionOlap (:395-435): DegreeCounter gives the
    group degree for the partitioned vertices and 1 for every person.  One more vertex cut
    whose canonical row is absent (its other representative rows stay) is joined by
    `ghost_degree` persons of group 0; it never executes, so nothing changes for them."""
    member, contain = es.user_edge_label(1), es.user_edge_label(2)
    sd = schema_dict([{"type_id": member, "multiplicity": MULTI}, {"type_id": contain, "multiplicity": MULTI}], [])
    edges, groups, group_of = [], [], []
    v = 0
    for deg in group_degrees:
        g = v
        groups.append(g)
        group_of.append(-1)
        v += 1
        for _ in range(deg):
            edges.append((v, g, member, []))
            edges.append((g, v, contain, []))
            group_of.append(g)
            v += 1
    ghost = v
    group_of.append(-2)
    v += 1
    for k in range(ghost_degree):
        edges.append((groups[0] + 1 + k, ghost, member, []))
    spec = es.GraphSpec(n=v, edges=edges, partitioned=groups + [ghost], pv_ghost=[ghost])
    rows, vids = es.build_rows(spec, oracle_schema(sd))
    live = [i for i in range(v) if i != ghost]
    degree1 = [group_degrees[groups.index(i)] if i in groups else 1 for i in live]
    # bothE BFS from group 0: the group, then its members
    bfs_g0 = [0 if i == groups[0] else (1 if group_of[i] == groups[0] else -1) for i in live]
    save("partition_groups", rows, vids[live], sd, degree1=np.asarray(degree1, np.int64),
         bfs_both_group0=np.asarray(bfs_g0, np.int64), group_index=np.asarray([live.index(g) for g in groups]),
         ghost_vid=np.int64(vids[ghost]))


if __name__ == "__main__":
    make_gotg()
    make_pagerank_tree()
    make_sssp_tree()
    make_degree_random(200, "degree_random", seed=7)
    make_degree_random(100, "degree_random100", seed=11)
    make_partition_groups()
    print("fixtures written to", HERE)
