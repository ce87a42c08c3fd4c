"""titan_amd — MI355X-native OLAP traversal engine for Titan (Fulgora GraphComputer path).

Compute runs in libtitan_gpu_olap.so (hand-written HIP for gfx950, C-ABI in
include/titan_gpu_olap.h).  This package is the host-side mirror of the reference's
TitanGraphComputer API plus a thin ctypes binding; it has no CPU fallback.
"""
from .engine import Engine, Rows, Schema, TitanException, rmat_edges, pick_roots, synth_rows  # noqa: F401
from .computer import (  # noqa: F401
    DegreeCounter, DegreeMapper, ExecutionException, GpuGraph, GpuGraphComputer, KeyValue,
    PageRankMapReduce, PageRankVertexProgram, ShortestDistanceMapReduce,
    ShortestDistanceVertexProgram, TitanGraphComputer,
)
from .generic import (  # noqa: F401
    ComputeKeyMapReduce, EdgeExpr, FulgoraMemory, GenericVertexProgram, MessageScope, Messenger, Vertices,
)
from .traversal import TraversalVertexProgram  # noqa: F401
from . import _lib  # noqa: F401

__all__ = [
    "Engine", "Rows", "Schema", "synth_rows", "TitanException", "rmat_edges", "pick_roots", "DegreeCounter", "DegreeMapper",
    "ExecutionException", "GpuGraph", "GpuGraphComputer", "KeyValue", "PageRankMapReduce",
    "PageRankVertexProgram", "ShortestDistanceMapReduce", "ShortestDistanceVertexProgram",
    "TitanGraphComputer", "ComputeKeyMapReduce", "FulgoraMemory", "GenericVertexProgram", "MessageScope",
    "Messenger", "Vertices", "EdgeExpr", "TraversalVertexProgram",
]
