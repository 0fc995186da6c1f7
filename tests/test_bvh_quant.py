"""Quantized 4-wide BVH nodes (pm_build.h quantize_bvh4, 64 B per node): the
encoder's boxes must contain the float boxes after the device's float decode,
so the culling test stays conservative and closest hits are unchanged (the
GPU side: test_gpu_parity scene tests on the soup / figure scenes, which
traverse the quantized nodes). CPU only: compiles a small checker against
pm_build.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cuda-raytrace_amd", "csrc")


@pytest.mark.parametrize("nprims,mode", [(1, ""), (7, ""), (50000, ""), (7, "refs"), (50000, "refs"), (1, "bigleaf")])
def test_quantized_boxes_contain_float_boxes(tmp_path, nprims, mode):
    """boxes contain the float boxes; with refs, LEAF_TRIS codes exactly the
    all-triangle leaves (~first storage slot); a leaf of >= LEAF_TRIS
    primitives is rejected (the scene then keeps the binary traversal)."""
    exe = tmp_path / "qcheck"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-ffp-contract=off", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "bvh4_quant_check.cpp"), os.path.join(CSRC, "pm_build.cpp"),
                    "-o", str(exe)], check=True, timeout=300)
    r = subprocess.run([str(exe), str(nprims)] + ([mode] if mode else []), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad 0" in r.stdout


def test_threaded_build_is_the_serial_tree(tmp_path):
    """The SAH build bins large ranges and builds left subtrees in threads
    (PM_BUILD_THREADS / OMP_NUM_THREADS): the binary nodes, refs and the
    quantized 4-wide nodes are bit-identical to the single-threaded build."""
    exe = tmp_path / "bcheck"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-ffp-contract=off", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "bvh_build_check.cpp"), os.path.join(CSRC, "pm_build.cpp"),
                    "-o", str(exe)], check=True, timeout=300)
    outs = []
    for t in ("1", "4"):
        r = subprocess.run([str(exe), "200000"], capture_output=True, text=True, timeout=300,
                           env={**os.environ, "PM_BUILD_THREADS": t})
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1] and "hash" in outs[0]


@pytest.mark.parametrize("radius", ["1", "3", "8"])
def test_ploc_host_tree_is_valid_and_thread_independent(tmp_path, radius):
    """pm_build.cpp build_ploc (the device builder's host restatement,
    csrc/pm_bvh_gpu.hip): a valid binary tree over every primitive in Morton
    order, internal boxes the exact unions of their children, the 4-wide
    collapse quantizable — and the same tree for 1 and 4 threads (only the
    nearest-neighbour search runs in parallel)."""
    exe = tmp_path / "pcheck"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-ffp-contract=off", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "ploc_check.cpp"), os.path.join(CSRC, "pm_build.cpp"),
                    "-o", str(exe)], check=True, timeout=300)
    outs = []
    for t in ("1", "4"):
        r = subprocess.run([str(exe), "60000", radius], capture_output=True, text=True, timeout=300,
                           env={**os.environ, "PM_BUILD_THREADS": t})
        assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1]
