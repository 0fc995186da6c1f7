"""CPU-only checks of the drop-in boundary: libpmhip.so loads, exports every
symbol include/pm_api.h declares, its POD layouts match the reference's, the
host-only entry points agree with the oracle, and the product library does
not link the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from pmrender.abi import PHOTON_DTYPE, RECORD_DTYPE, RenderParams, Stats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pm_api.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("pm_create", "pm_destroy", "pm_render", "pm_add_trimesh", "pm_add_sphere", "pm_add_disk",
                 "pm_add_light_disk", "pm_trace_photons", "pm_build_photon_map", "pm_gather", "pm_final"):
        assert must in names
    assert len(names) >= 40


def test_library_exports_every_declared_symbol(hip_mod):
    lib = hip_mod.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"undefined exports: {missing}"


def test_exports_are_c_linkage():
    lib = os.path.join(ROOT, "cuda-raytrace_amd", "lib", "libpmhip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for n in declared_functions():
        assert n in exported, f"{n} not exported with C linkage"


def test_product_does_not_link_the_oracle():
    lib = os.path.join(ROOT, "cuda-raytrace_amd", "lib", "libpmhip.so")
    deps = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True).stdout
    assert "liborc" not in deps
    syms = subprocess.run(["nm", "-D", lib], capture_output=True, text=True, check=True).stdout
    assert "orc_" not in syms


def test_pod_layouts(tmp_path):
    """ctypes / numpy mirrors == the C compiler's view of include/pm_api.h."""
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "pm_api.h"\nint main(void){printf("%zu %zu %zu %zu %zu %zu",'
                   'sizeof(pm_photon), sizeof(pm_record), sizeof(pm_render_params), sizeof(pm_stats),'
                   'offsetof(pm_render_params, paths_per_pass), offsetof(pm_render_params, gather_structure));'
                   'printf(" %zu %zu %zu", sizeof(pm_config), offsetof(pm_config, n_devices), offsetof(pm_config, devices));'
                   'return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    from pmrender.abi import PMConfig
    assert got == [PHOTON_DTYPE.itemsize, RECORD_DTYPE.itemsize, ctypes.sizeof(RenderParams), ctypes.sizeof(Stats),
                   RenderParams.paths_per_pass.offset, RenderParams.gather_structure.offset,
                   ctypes.sizeof(PMConfig), PMConfig.n_devices.offset, PMConfig.devices.offset]
    assert ctypes.sizeof(PMConfig) == 32         # the round-2 pm_config size (int device + 7 reserved ints)
    assert PHOTON_DTYPE.itemsize == 40           # CudaPhoton, photonmapping.h:32-41


def test_default_params_match_c(hip_mod):
    lib = hip_mod.load_library()
    p = RenderParams()
    lib.pm_default_params(ctypes.byref(p))
    q = RenderParams.defaults()
    for name, _ in RenderParams._fields_:
        if name != "reserved":
            assert getattr(p, name) == pytest.approx(getattr(q, name)), name
    assert (p.paths_per_pass, p.max_photon_count, p.rng_seed) == (262144, 4, 777)


def test_halton_permutation_equals_oracle(hip_mod, oracle_mod):
    for seed in (0, 1, 2, 5489, 123456):
        assert np.array_equal(hip_mod.halton_permutation(seed), oracle_mod.halton_permutation(seed))


def test_host_kdtree_equals_oracle(hip_mod, oracle_mod):
    """pm_kdtree_build_host (reference CreatePhotonMap layout) == oracle, bit for bit."""
    from test_oracle_kat import _random_photons
    for n, seed in ((1, 0), (2, 1), (7, 2), (5000, 3)):
        ph = _random_photons(n, seed, valid_frac=1.0 if n < 8 else 0.7)
        a = hip_mod.kdtree_build_host(ph)
        b = oracle_mod.Oracle.build_kdtree(ph)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_host_kdtree_on_traced_photons(hip_mod, oracle_mod):
    from pmrender import scenes
    orc = scenes.cornell_box(16, 16).load_into(oracle_mod.Oracle(nthreads=2))
    slots = orc.trace_photons(RenderParams.defaults(paths_per_pass=8192))
    a = hip_mod.kdtree_build_host(slots)
    b = oracle_mod.Oracle.build_kdtree(slots)
    assert len(a) == (slots["bits"] & 1).sum()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_create_reports_error_without_device(hip_mod):
    """No GPU in the build container: pm_create must fail with a message, not crash."""
    lib = hip_mod.load_library()
    h = ctypes.c_void_p()
    rc = lib.pm_create(ctypes.byref(h), None)
    if rc == 0:
        lib.pm_destroy(h)
        pytest.skip("a HIP device is present")
    assert rc == 2 and b"HIP" in lib.pm_last_error(None)
