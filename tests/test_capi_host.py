"""CPU-side checks of the C-ABI library (no GPU needed).

* libsm_hip.so loads and exports every function include/sm_hip.h declares;
* the host-only helpers behave: shard plan (include/mpi_setup.h:6-23 rules),
  the synthetic field generator reproduces the golden inputs bit for bit, the
  28-byte gauge-conf format round-trips (src/gauge_conf.cpp:378-423, 495-546);
* without a GPU every device entry point fails loudly (no CPU fallback).
"""
import ctypes
import os
import re
import struct
import subprocess

import numpy as np
import pytest

from conftest import REPO, bits_equal, fixture_names, load_fixture, planes

sm = pytest.importorskip("schwingermodel_amd")
lib = sm.lib


def declared_functions():
    with open(os.path.join(REPO, "include", "sm_hip.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sm_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n


def test_library_is_gfx950_code_object():
    with open(sm._lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_shard_plan():
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    assert lib.sm_shard_plan(4096, 8, 3, ctypes.byref(t0), ctypes.byref(Wt)) == 0
    assert (t0.value, Wt.value) == (1536, 512)
    assert lib.sm_shard_plan(100, 8, 0, ctypes.byref(t0), ctypes.byref(Wt)) != 0
    assert b"divisible" in lib.sm_last_error()
    assert lib.sm_shard_plan(64, 2, 2, None, None) != 0


@pytest.mark.parametrize("name", fixture_names())
def test_generator_reproduces_golden_inputs(name):
    meta, a = load_fixture(name)
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    U = np.empty(4 * S)
    u0, u1 = planes(U, S)
    lib.sm_fill_gauge(4321, meta["sigma"], Nt, 0, Nx, 0, Nt, u0.ctypes.data, u1.ctypes.data)
    assert bits_equal(U, a["U"])
    P = np.empty(4 * S)
    p0, p1 = planes(P, S)
    lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, p0.ctypes.data, p1.ctypes.data)
    assert bits_equal(P, a["psi"])


def test_generator_shards_tile_the_global_field():
    Nx, Nt, P = 16, 24, 4
    S = Nx * Nt
    g0 = np.empty(2 * S)
    g1 = np.empty(2 * S)
    lib.sm_fill_gauge(7, 0.3, Nt, 0, Nx, 0, Nt, g0.ctypes.data, g1.ctypes.data)
    G = g0.view(np.complex128).reshape(Nx, Nt)
    Wt = Nt // P
    for s in range(P):
        b0 = np.empty(2 * Nx * Wt)
        b1 = np.empty(2 * Nx * Wt)
        lib.sm_fill_gauge(7, 0.3, Nt, 0, Nx, s * Wt, Wt, b0.ctypes.data, b1.ctypes.data)
        assert np.array_equal(b0.view(np.complex128).reshape(Nx, Wt), G[:, s * Wt:(s + 1) * Wt])


def test_gauge_conf_binary_format(tmp_path):
    meta, a = load_fixture("l8x8_hot_m0p2")
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    u0, u1 = planes(a["U"], S)
    path = str(tmp_path / "2D_U1_Ns8_Nt8_b20000_m02000_0.ctxt")
    assert lib.sm_conf_write(path.encode(), Nx, Nt, u0.ctypes.data, u1.ctypes.data) == 0
    raw = open(path, "rb").read()
    assert len(raw) == Nx * Nt * 2 * 28  # 28-byte packed records, no padding
    # record k = (x, t, mu) in x-outer, t, mu-inner order
    x, t, mu, re_, im = struct.unpack_from("<iiidd", raw, 28 * (2 * (3 * Nt + 5) + 1))
    assert (x, t, mu) == (3, 5, 1)
    n = 3 * Nt + 5
    assert (re_, im) == (u1[2 * n], u1[2 * n + 1])
    back = np.empty(4 * S)
    b0, b1 = planes(back, S)
    assert lib.sm_conf_read(path.encode(), Nx, Nt, b0.ctypes.data, b1.ctypes.data) == 0
    assert bits_equal(back, a["U"])
    assert lib.sm_conf_read(str(tmp_path / "missing").encode(), Nx, Nt, b0.ctypes.data, b1.ctypes.data) != 0


@pytest.mark.parametrize("name", ["conf8x8_hot", "conf32x48_b3"])
def test_conf_io_matches_reference_saveconf(tmp_path, name):
    """Pinned to the reference itself: tests/golden/<name>.ctxt was written by
    the reference's SaveConf (src/gauge_conf.cpp:378-423; conf32x48 on 2x2 MPI
    ranks, through its MPI_Gatherv displacements) from the fixture's U, and
    ref_conf_read is what its GaugeConf::readBinary (:495-546) read back.
    sm_conf_write must produce the same bytes, sm_conf_read the same field."""
    import hashlib
    import json
    from conftest import GOLDEN
    meta = json.load(open(os.path.join(GOLDEN, "manifest.json")))["conf"][name]
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    with np.load(os.path.join(GOLDEN, meta["file"]), allow_pickle=False) as z:
        U, read_back = z["U"].copy(), z["ref_conf_read"].copy()
    ref_bytes = open(os.path.join(GOLDEN, meta["ctxt"]), "rb").read()
    assert hashlib.sha256(ref_bytes).hexdigest() == meta["sha256"]
    u0, u1 = planes(U, S)
    path = str(tmp_path / "conf.ctxt")
    assert lib.sm_conf_write(path.encode(), Nx, Nt, u0.ctypes.data, u1.ctypes.data) == 0
    assert open(path, "rb").read() == ref_bytes
    back = np.empty(4 * S)
    b0, b1 = planes(back, S)
    assert lib.sm_conf_read(os.path.join(GOLDEN, meta["ctxt"]).encode(), Nx, Nt, b0.ctypes.data,
                            b1.ctypes.data) == 0
    assert bits_equal(back, read_back) and bits_equal(back, U)


def test_no_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    h = ctypes.c_void_p()
    rc = lib.sm_create(ctypes.byref(h), 8, 8, 1, 0, 0, None)
    assert rc != 0 and h.value is None
    with pytest.raises(sm.SMError):
        sm.init(8, 8)


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of the ABI structs have the C header's size and offsets."""
    import schwingermodel_amd._lib as L
    structs = {"sm_cg_result": L.CGResult, "sm_hmc_params": L.HMCParams,
               "sm_hamiltonian_terms": L.HamiltonianTerms, "sm_hmc_result": L.HMCResult,
               "sm_hmc_summary": L.HMCSummary}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sm_hip.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {tuple(ln.split()[:2]): int(ln.split()[2]) for ln in out if ln}
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_jackknife_matches_reference():
    """sm_jackknife_error == the reference's Jackknife_error(dat, 20) bit for bit
    (golden values from src/statistics.cpp via make_golden.py), including its
    integer binning for series shorter than / not a multiple of 20."""
    import json
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
        cases = json.load(f)["jackknife"]
    for c in cases:
        d = np.array(c["data"])
        got = sm.lib.sm_jackknife_error(d.ctypes.data, len(d), c["bin"])
        assert got == c["jackknife_error"], (len(d), got, c["jackknife_error"])


def test_conf_read_truncated_file_fails(tmp_path):
    """A conf file shorter than Nx*Nt*2 records fails with SM_ERR_ARG and a
    message naming the site (sm_conf.cpp). The reference's readBinary does not
    check its reads (src/gauge_conf.cpp:515-531), so past the end it would keep
    whatever the variables held; the drop-in refuses instead."""
    Nx, Nt = 4, 4
    S = Nx * Nt
    u = np.arange(4 * S, dtype=np.float64)
    u0, u1 = planes(u, S)
    path = str(tmp_path / "short.ctxt")
    assert lib.sm_conf_write(path.encode(), Nx, Nt, u0.ctypes.data, u1.ctypes.data) == 0
    with open(path, "r+b") as f:
        f.truncate(28 * (2 * S - 3))
    back = np.empty(4 * S)
    b0, b1 = planes(back, S)
    assert lib.sm_conf_read(path.encode(), Nx, Nt, b0.ctypes.data, b1.ctypes.data) == 1
    assert b"truncated" in lib.sm_last_error()


def test_placement_probe_setting_is_validated():
    """sm_set_placement_probe takes 0 (no probe) .. 8 candidates per buffer and
    rejects anything else without touching the current setting (sm_place.cpp);
    sm_get_placement_probe reads it, so the test restores what it found."""
    before = lib.sm_get_placement_probe()
    assert 0 <= before <= 8
    try:
        for bad in (-1, 9, 100):
            assert lib.sm_set_placement_probe(bad) == 1
            assert b"0..8" in lib.sm_last_error()
            assert lib.sm_get_placement_probe() == before
        for ok in (0, 8, 5):
            assert lib.sm_set_placement_probe(ok) == 0
            assert lib.sm_get_placement_probe() == ok
    finally:
        assert lib.sm_set_placement_probe(before) == 0


def test_placement_buffer_names():
    """Bit i of sm_placement_report's mask names buffer i of the probe's
    search order (one table in sm_place.cpp serves the probe and this call)."""
    names = [lib.sm_placement_buffer_name(i) for i in range(5)]
    assert names == [b"x", b"d1", b"d0", b"d2", None]
    assert lib.sm_placement_buffer_name(-1) is None


def test_comm_info_null_context():
    """sm_comm_info refuses a null context and writes nothing (no GPU needed)."""
    t, n, r = ctypes.c_int(-7), ctypes.c_int(-7), ctypes.c_int(-7)
    assert lib.sm_comm_info(None, ctypes.byref(t), ctypes.byref(n), ctypes.byref(r)) == 1
    assert (t.value, n.value, r.value) == (-7, -7, -7)
