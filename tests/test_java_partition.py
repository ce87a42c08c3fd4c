"""CPU: the Java multi-GPU host logic where no JDK exists (nothing compiled or ran
PartitionedRun).  The parts that decide results are restated here and pinned:

* PartitionedRun.blockRanges — contiguous scan-block ranges balanced by rows + entries — is
  transliterated line for line (java_block_ranges) and checked against the Java source's own
  formula text, against titan_amd.distributed.balanced_row_ranges (the same rule over rows;
  one-row blocks must give identical cuts) and against the properties the workers rely on
  (contiguous, covering, possibly-empty ranges, balance within one block).
* The worker protocol's result placement (ids from tgo_vertex_ids, the first `live` values of
  each worker, worker-major) is what tests/test_gpu_distributed.py RowRanks runs on the GPU.
* Every class of the Java host layer referenced from another package is imported (a missing
  import of PartitionedRun in GpuGraphComputer went unnoticed without a compiler).
"""
import os
import re

import numpy as np
import pytest

from titan_amd.distributed import balanced_row_ranges

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "main", "java")
PRUN = os.path.join(JAVA, "com", "thinkaurelius", "titan", "graphdb", "olap", "gpu", "PartitionedRun.java")


def java_block_ranges(weights, world):
    """PartitionedRun.blockRanges, statement for statement (long arithmetic, >>> 1 midpoint)."""
    nb = len(weights)
    prefix = [0] * (nb + 1)
    for i in range(nb):
        prefix[i + 1] = prefix[i] + int(weights[i])
    total = prefix[nb]
    cut = [0] * (world + 1)
    for r in range(1, world):
        target = (total * r + world - 1) // world
        lo, hi = 0, nb
        while lo < hi:
            mid = (lo + hi) >> 1
            if prefix[mid] < target:
                lo = mid + 1
            else:
                hi = mid
        cut[r] = max(cut[r - 1], min(nb, lo))
    cut[world] = nb
    return cut


def test_transliteration_matches_the_java_source():
    src = open(PRUN).read()
    body = src[src.index("static int[] blockRanges("):src.index("// ------------------------------------------------------------------ partition + run")]
    for stmt in ("prefix[i + 1] = prefix[i] + weights[i];", "final long target = (total * r + world - 1) / world;",
                 "int mid = (lo + hi) >>> 1;", "if (prefix[mid] < target) lo = mid + 1; else hi = mid;",
                 "cut[r] = Math.max(cut[r - 1], Math.min(nb, lo));", "cut[world] = nb;"):
        assert stmt in body, stmt
    # the block weight the ranges balance: rows + entries of the block
    assert "long weight() { return keys.length + entryBegin[keys.length]; }" in src


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8, 13])
def test_block_ranges_properties(seed, world):
    rng = np.random.default_rng(seed)
    nb = int(rng.integers(0, 40))
    w = rng.integers(1, 1000, nb) * (rng.random(nb) < 0.9)       # some empty blocks
    if nb and seed % 2:
        w[rng.integers(0, nb)] = 100000                           # a hub's block
    cut = java_block_ranges(w, world)
    assert len(cut) == world + 1 and cut[0] == 0 and cut[-1] == nb
    assert all(a <= b for a, b in zip(cut, cut[1:]))              # contiguous, possibly empty
    total = int(np.sum(w))
    prefix = np.concatenate([[0], np.cumsum(w)])
    for r in range(1, world):                                     # the first boundary reaching r / world
        target = -(-total * r // world)
        assert prefix[cut[r]] >= target or cut[r] == nb
        assert cut[r] == cut[r - 1] or prefix[cut[r] - 1] < target
    big = int(np.max(w)) if nb else 0
    for r in range(world):                                        # balanced within one block
        assert prefix[cut[r + 1]] - prefix[cut[r]] <= -(-total // world) + big


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_one_row_blocks_equal_balanced_row_ranges(world):
    """With one row per block the Java rule and distributed.balanced_row_ranges cut the same rows."""
    rng = np.random.default_rng(world)
    deg = rng.integers(0, 50, 500)
    deg[7] = 5000
    eb = np.concatenate([[0], np.cumsum(deg)])
    cut = java_block_ranges(1 + deg, world)
    assert [(cut[r], cut[r + 1]) for r in range(world)] == balanced_row_ranges(eb, world)


def test_cross_package_classes_are_imported():
    files = {}
    for dirpath, _, names in os.walk(JAVA):
        for n in names:
            if n.endswith(".java"):
                p = os.path.join(dirpath, n)
                files[p] = open(p).read()
    pkg_of, classes = {}, {}
    for p, src in files.items():
        pkg = re.search(r"^package\s+([\w.]+);", src, re.M).group(1)
        pkg_of[p] = pkg
        for c in re.findall(r"^public\s+(?:final\s+|abstract\s+)*class\s+(\w+)", src, re.M):
            classes[c] = pkg
    for p, src in files.items():
        code = re.sub(r"/\*.*?\*/|//[^\n]*", "", src, flags=re.S)
        for c, pkg in classes.items():
            if pkg == pkg_of[p] or not re.search(r"\b" + c + r"\b", code):
                continue
            assert re.search(r"^import\s+" + re.escape(pkg + "." + c) + r";", src, re.M), (os.path.basename(p), c)
