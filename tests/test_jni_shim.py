"""CPU: the Java host layer's native boundary where no JDK exists.

* java/jni/titan_gpu_olap_jni.c is compiled with gcc -fsyntax-only against the REAL C-ABI
  header (include/titan_gpu_olap.h) and a minimal JNI declaration file (tests/jni_stub/jni.h,
  the JNI specification's signatures), so a drift between the shim and the C-ABI fails here.
* Every `native` method of TgoNative.java has exactly one JNI entry point in the shim, and
  the Java side calls the natives and helpers it relies on with the visibility it needs.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "java", "jni", "titan_gpu_olap_jni.c")
JAVA = os.path.join(ROOT, "java", "src", "main", "java", "com", "thinkaurelius", "titan", "graphdb", "olap")
NATIVE = os.path.join(JAVA, "gpu", "TgoNative.java")
COMPUTER = os.path.join(JAVA, "computer", "GpuGraphComputer.java")
SCANJOB = os.path.join(JAVA, "gpu", "CsrCollectingScanJob.java")


def _read(p):
    with open(p) as f:
        return f.read()


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_shim_type_checks_against_the_c_abi():
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"), SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_method_has_one_entry_point():
    java = _read(NATIVE)
    natives = re.findall(r"\bnative\s+[\w\[\]<>]+\s+(\w+)\s*\(", java)
    shim = re.findall(r"JNIEXPORT\s+\w+\s+JNICALL\s+JFN\((\w+)\)", _read(SHIM))
    assert natives and sorted(natives) == sorted(shim)
    assert len(set(shim)) == len(shim)


def test_helpers_called_across_packages_are_public():
    """GpuGraphComputer (package ...olap.computer) calls TgoNative.check / checked (package
    ...olap.gpu): package-private helpers would not compile."""
    java = _read(NATIVE)
    for name in ("check", "checked"):
        assert re.search(r"public\s+static\s+[\w<> ]*\b" + name + r"\s*\(", java), name
    comp = _read(COMPUTER)
    assert "TgoNative.check(" in comp and "TgoNative.checked(" in comp


def test_computer_follows_fulgora_iteration_and_result_modes():
    """Fulgora increments the iteration after every superstep 0..T (FulgoraGraphComputer.java:
    181-188) and complete() steps back once (FulgoraMemory.java:73-76): T + 1 increments.  Unset
    modes come from the program (GraphComputerHelper.getPersistState / getResultGraphState)."""
    comp = _read(COMPUTER)
    assert re.search(r"for \(int i = 0; i <= program\.iterations\(\); i\+\+\) memory\.incrIteration\(\);", comp)
    assert "GraphComputerHelper.getPersistState(Optional.ofNullable(vertexProgram)" in comp
    assert "GraphComputerHelper.getResultGraphState(Optional.ofNullable(vertexProgram)" in comp
    assert "handle.rethrowFailure();" in comp.split("TgoNative.finishLoad(ctx)")[0]


def test_scan_job_failures_are_sticky():
    job = _read(SCANJOB)
    assert "public void rethrowFailure()" in job
    assert re.search(r"if \(handle\.failure == null\) handle\.failure = e;", job)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_load_csr_validates_array_lengths_before_pinning(tmp_path):
    """loadCsr hands tgo_load_csr the pinned Java arrays, which stages out_off[n] /
    in_off[n] entries from them — short or null index / weight arrays must fail with
    TGO_E_INVALID before the C-ABI is reached (tests/jni_harness.c: a fake JNIEnv, the shim
    linked against the harness's recording tgo_load_csr and the real library for the rest)."""
    exe = _build_harness(tmp_path)
    run = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert run.returncode == 0, run.stdout + run.stderr
    assert run.stdout.count("ok  ") == 27, run.stdout


def _build_harness(tmp_path):
    lib = os.path.join(ROOT, "titan_amd")
    if not os.path.exists(os.path.join(lib, "libtitan_gpu_olap.so")):
        pytest.skip("libtitan_gpu_olap.so not built")
    exe = str(tmp_path / "jni_harness")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "jni_harness.c"), SHIM, "-o", exe,
                        "-L", lib, "-ltitan_gpu_olap", "-Wl,-rpath," + lib, "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.gpu
@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_java_multi_gpu_natives_world1(tmp_path):
    """the Java multi-GPU path's natives (TgoNative.partLayout /
    loadPartition / exchangeRcclId / exchangeRcclCreate / partSsspRun / partPageRankRun /
    partBfsRun / partMsbfsRun / partMsLevels — what PartitionedRun calls per worker) run through
    the JNI shim against the real library at world 1 over RCCL, and equal the one-GPU engine on
    the same graph (SSSP and BFS bit-exact, PageRank in both exchange modes within 1e-12 L1); and
    (round 6) the row path PartitionedRun now takes — loadRows blocks, the collective
    finishPartitionRows, partSsspRun / partPageRankRun / partWeightMin — on synthetic edgestore
    rows that are ALL cut at a hard limit of 3, against tgo_load_rows on one GPU."""
    exe = _build_harness(tmp_path)
    run = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "FAIL" not in run.stdout and run.stdout.count("ok  ") == 27 + 13 + 7, run.stdout
