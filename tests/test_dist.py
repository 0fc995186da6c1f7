"""World-size-2..8 gloo tests of the multi-GPU pass runner (pmrender/dist.py) on
CPU: the same PassRunner that bench.py drives over RCCL, here over gloo with
an oracle-backed engine. Checks both photon exchanges against a
single-process run over the same global paths."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from pmrender.abi import PHOTON_DTYPE, RECORD_DTYPE, RenderParams  # noqa: E402

PATHS = 4096  # per rank


class OracleEngine:
    """PassRunner engine on the CPU oracle (test infrastructure only)."""
    FX = 2.0 ** 12  # fixed-point scale of the int64 partials

    def __init__(self, scene, params):
        import oracle
        self.oracle = oracle
        self.orc = scene.load_into(oracle.Oracle(nthreads=2))
        self.init = self.orc.eye_pass(params)
        self.recs = self.init.copy()
        self.slots = None
        self.slot_buf = None
        self.nodes = None
        self.view = None      # active-record view (indices), like pm_set_record_view

    def num_records(self):
        return len(self.recs)

    def alloc(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype)

    def use_slot_buffer(self, t):
        self.slot_buf = t

    def reset_records(self, p):
        self.recs = self.init.copy()

    def set_record_view(self, active_only=True):
        self.view = np.nonzero((self.recs["flags"] & 7) == 0)[0] if active_only else None
        return len(self.view) if active_only else len(self.recs)

    def _rec(self, i):
        return int(self.view[i]) if self.view is not None else int(i)

    def trace_photons(self, p, pass_index, path_begin, path_count, slot_path_base):
        s = self.orc.trace_photons(p, pass_index, path_begin, path_count)
        if self.slot_buf is None:
            self.slots = s
            return
        off = (path_begin - slot_path_base) * p.max_photon_count * PHOTON_DTYPE.itemsize
        self.slot_buf.numpy()[off:off + s.nbytes] = s.view(np.uint8)

    def build_photon_map(self, p, n_slots):
        if self.slot_buf is None:
            src = self.slots[:n_slots]
        else:
            src = np.frombuffer(self.slot_buf.numpy()[: n_slots * PHOTON_DTYPE.itemsize].tobytes(), PHOTON_DTYPE)
        self.nodes = self.oracle.Oracle.build_kdtree(src)

    def gather(self, p):
        self.orc.gather(self.nodes, self.recs, p)

    def gather_range(self, p, b, n):
        sub = self.recs[b:b + n].copy()
        self.orc.gather(self.nodes, sub, p)
        self.recs[b:b + n] = sub

    def gather_partial(self, p, out):
        part = self.orc.gather_partial(self.nodes, self.recs)
        if self.view is not None:
            part = part[self.view]
        n = len(part)
        out[:n, 0] = torch.from_numpy(part[:, 0].astype(np.int64))
        out[:n, 1:] = torch.from_numpy(np.rint(part[:, 1:].astype(np.float64) * self.FX).astype(np.int64))

    def ppm_update(self, p, partial, b, n):
        import ctypes
        lib = self.oracle.load()
        P = partial.numpy()
        for i in range(n):
            ri = self._rec(b + i)
            r = self.recs[ri]
            if r["flags"] & 7:
                continue
            r2 = np.float32([r["radius2"]])
            N = np.float32([r["photon_count"]])
            flux = np.ascontiguousarray(r["flux"], np.float32)
            L = (P[i, 1:].astype(np.float64) / self.FX).astype(np.float32)
            fp = ctypes.POINTER(ctypes.c_float)
            lib.orc_ppm_update(r2.ctypes.data_as(fp), N.ctypes.data_as(fp), flux.ctypes.data_as(fp), int(P[i, 0]),
                               L.ctypes.data_as(fp), float(p.ppm_alpha))
            self.recs[ri]["radius2"], self.recs[ri]["photon_count"] = r2[0], N[0]
            self.recs[ri]["flux"] = flux

    def gather_split(self, p, count, flux):
        part = self.orc.gather_partial(self.nodes, self.recs)
        if self.view is not None:
            part = part[self.view]
        n = len(part)
        count[:n] = torch.from_numpy(part[:, 0].astype(np.int32))
        flux[:n] = torch.from_numpy(np.rint(part[:, 1:].astype(np.float64) * self.FX).astype(np.int64))

    def ppm_update_split(self, p, count, flux_chunk, v_begin, v_count):
        """every view record's radius / photon count from the global counts;
        flux from the summed chunk for [v_begin, v_begin + v_count) only"""
        import ctypes
        lib = self.oracle.load()
        fp = ctypes.POINTER(ctypes.c_float)
        C, F = count.numpy(), flux_chunk.numpy()
        n_view = len(self.view) if self.view is not None else len(self.recs)
        for i in range(n_view):
            ri = self._rec(i)
            r = self.recs[ri]
            if r["flags"] & 7 or C[i] <= 0:
                continue
            r2 = np.float32([r["radius2"]])
            N = np.float32([r["photon_count"]])
            fl = np.ascontiguousarray(r["flux"], np.float32)
            own = v_begin <= i < v_begin + v_count
            L = (F[i - v_begin].astype(np.float64) / self.FX).astype(np.float32) if own else np.zeros(3, np.float32)
            lib.orc_ppm_update(r2.ctypes.data_as(fp), N.ctypes.data_as(fp), fl.ctypes.data_as(fp), int(C[i]),
                               L.ctypes.data_as(fp), float(p.ppm_alpha))
            self.recs[ri]["radius2"], self.recs[ri]["photon_count"] = r2[0], N[0]
            self.recs[ri]["flux"] = fl

    def get_radius2(self, b, n, out):
        idx = self.view[b:b + n] if self.view is not None else np.arange(b, b + n)
        out[:n] = torch.from_numpy(self.recs["radius2"][idx].copy())

    def set_radius2(self, src, b, n):
        idx = self.view[b:b + n] if self.view is not None else np.arange(b, b + n)
        self.recs["radius2"][idx] = src[:n].numpy()

    def final(self, emitted, b, n, out):
        img = self.orc.final(self.recs, emitted)
        out.copy_(torch.from_numpy(img[b:b + n]))

    def final_view(self, emitted, b, n, out):
        img = self.orc.final(self.recs, emitted)
        out[:n] = torch.from_numpy(img[self.view[b:b + n]])

    def record_view_list(self, out):
        out.copy_(torch.from_numpy(self.view.astype(np.int32)))


class OracleEngineLate(OracleEngine):
    """The two-phase update of HipEngine (pm_ppm_update_split_radius /
    _flux): radii and photon counts from the global counts before the next
    gather, the owner's flux after it. Each flux update replays the oracle's
    ppm_update from the record's state before its radius update, so the
    arithmetic is the oracle's own."""

    def __init__(self, scene, params):
        super().__init__(scene, params)
        self.pending = {}   # view index -> (radius2, photon_count, M) before the radius update

    def reset_records(self, p):
        super().reset_records(p)
        self.pending = {}   # the reset discards the pass whose flux is still in flight

    def ppm_update_radius(self, p, count, ratio):
        import ctypes
        lib = self.oracle.load()
        fp = ctypes.POINTER(ctypes.c_float)
        C, Q = count.numpy(), ratio.numpy()
        n_view = len(self.view) if self.view is not None else len(self.recs)
        self.pending = {}
        for i in range(n_view):
            r = self.recs[self._rec(i)]
            Q[i] = -1.0
            if r["flags"] & 7 or C[i] <= 0:
                continue
            r2 = np.float32([r["radius2"]])
            N = np.float32([r["photon_count"]])
            self.pending[i] = (r2[0], N[0], int(C[i]))
            fl = np.zeros(3, np.float32)
            lib.orc_ppm_update(r2.ctypes.data_as(fp), N.ctypes.data_as(fp), fl.ctypes.data_as(fp), int(C[i]),
                               np.zeros(3, np.float32).ctypes.data_as(fp), float(p.ppm_alpha))
            r["radius2"], r["photon_count"] = r2[0], N[0]
            Q[i] = 1.0

    def ppm_update_flux(self, p, ratio, flux_chunk, v_begin, v_count):
        import ctypes
        lib = self.oracle.load()
        fp = ctypes.POINTER(ctypes.c_float)
        F = flux_chunk.numpy()
        for i in range(v_begin, v_begin + v_count):
            if i not in self.pending:
                continue
            r2o, No, M = self.pending[i]
            ri = self._rec(i)
            r2 = np.float32([r2o])
            N = np.float32([No])
            fl = np.ascontiguousarray(self.recs[ri]["flux"], np.float32)
            L = (F[i - v_begin].astype(np.float64) / self.FX).astype(np.float32)
            lib.orc_ppm_update(r2.ctypes.data_as(fp), N.ctypes.data_as(fp), fl.ctypes.data_as(fp), M,
                               L.ctypes.data_as(fp), float(p.ppm_alpha))
            self.recs[ri]["flux"] = fl


def _scene():
    from pmrender import scenes
    sc = scenes.cornell_box(40, 24)
    sc.camera = scenes.rays_from_pinhole(sc)
    return sc


def _worker(rank, world, port, exchange, outdir, total=None, late=False, reset_at=-1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cuda-raytrace_amd"), os.path.join(root, "oracle")]
    from pmrender.dist import PassRunner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=25.0)
    eng = (OracleEngineLate if late else OracleEngine)(_scene(), p)
    runner = PassRunner(eng, p, rank, world, exchange, force_exchange=world == 1, total_paths=total)
    assert runner.multi and (exchange != "reduce" or runner.late_flux == late)
    for pass_index in range(2):
        runner.step(pass_index, reset=pass_index == reset_at)
    runner.flush()
    out = torch.zeros((runner.n_records, 3), dtype=torch.float32)
    runner.final_gather(float(runner.emitted_per_pass * 2), out)
    assert runner.emitted_per_pass == (total if total is not None else PATHS * world)
    if exchange == "reduce":   # PPM state is owned per chunk of the active-record view
        owned = eng.view[runner.v_begin:runner.v_begin + runner.v_count]
    else:                      # the rank's interleaved 8-row bands
        owned = np.concatenate([np.arange(b, b + c) for b, c in runner.bands[rank]] + [np.zeros(0, np.int64)])
    np.save(os.path.join(outdir, f"idx{rank}.npy"), owned)
    np.save(os.path.join(outdir, f"recs{rank}.npy"), eng.recs[owned])
    np.save(os.path.join(outdir, f"img{rank}.npy"), out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _single_process_reference(world, total=None, reset_at=-1):
    """1 process, the union of all ranks' global paths, kd gather."""
    import oracle
    n = total if total is not None else PATHS * world
    p = RenderParams.defaults(paths_per_pass=n, initial_radius2=25.0)
    orc = _scene().load_into(oracle.Oracle(nthreads=2))
    recs = orc.eye_pass(p)
    init = recs.copy()
    for pass_index in range(2):
        if pass_index == reset_at:
            recs = init.copy()
        slots = orc.trace_photons(p, pass_index, 0, n)
        orc.gather(oracle.Oracle.build_kdtree(slots), recs, p)
    return recs, orc.final(recs, float(n * 2))


@pytest.mark.parametrize("exchange,world,total", [("allgather", 2, None), ("reduce", 2, None), ("reduce", 4, None),
                                                  ("allgather", 3, None), ("reduce", 1, None), ("allgather", 1, None),
                                                  ("reduce", 8, None), ("allgather", 8, None),
                                                  ("reduce", 3, 3 * PATHS + 1001), ("allgather", 3, 3 * PATHS + 1001),
                                                  ("allgather", 8, 8 * PATHS - 4093),
                                                  ("reduce", 4, 5), ("allgather", 8, 9)])
def test_two_rank_pass_matches_single_process(exchange, world, total, tmp_path):
    """world-size 2 (and 3 / 4 / 8: view chunks and bands that do not divide
    evenly; 8 = the production rank count of one node) over gloo vs one
    process over the same global paths; world 1 with the exchange path forced
    (force_exchange: what the GPU test runs on RCCL); `total`: strong scaling
    (bench.py --total-paths), a fixed path count split over the ranks with a
    short last chunk — or, for totals below the world size's chunks (4 ranks
    / 5 paths, 8 / 9), ranks with no paths at all"""
    mp.start_processes(_worker, args=(world, _free_port(), exchange, str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    ref_recs, ref_img = _single_process_reference(world, total)
    idx = np.concatenate([np.load(tmp_path / f"idx{r}.npy") for r in range(world)])
    recs = np.concatenate([np.load(tmp_path / f"recs{r}.npy") for r in range(world)]).view(RECORD_DTYPE)
    expect = np.nonzero((ref_recs["flags"] & 7) == 0)[0] if exchange == "reduce" else np.arange(len(ref_recs))
    assert np.array_equal(np.sort(idx), expect)        # every record owned exactly once
    ref_recs = ref_recs[idx]
    assert np.array_equal(recs["photon_count"], ref_recs["photon_count"])
    assert np.array_equal(recs["radius2"].view(np.uint32), ref_recs["radius2"].view(np.uint32))
    img = np.load(tmp_path / "img0.npy")
    for r in range(1, world):                                          # every rank holds the full image
        assert np.array_equal(img, np.load(tmp_path / f"img{r}.npy"))
    if exchange == "allgather":
        # replicated map over identical slots + canonical kd-tree: bit-exact
        assert np.array_equal(recs["flux"].view(np.uint32), ref_recs["flux"].view(np.uint32))
        assert np.array_equal(img.view(np.uint32), ref_img.view(np.uint32))
    else:
        # per-rank partial sums: exact M, flux within the fixed-point/fp32 rounding
        np.testing.assert_allclose(recs["flux"], ref_recs["flux"], rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(img, ref_img, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,unit,world", [(2_073_600, 240 * 64, 8), (3072, 8 * 64, 2), (100, 64, 4), (1, 512, 2)])
def test_allgather_bands_cover_every_record_once(n, unit, world):
    """All-gather mode ownership: 8-row bands dealt
    round-robin in runs, about four runs per rank, every record exactly once."""
    from pmrender.dist import _bands
    owned = _bands(n, unit, world)
    idx = np.concatenate([np.arange(b, b + c) for r in owned for b, c in r]) if n else np.zeros(0)
    assert np.array_equal(np.sort(idx), np.arange(n))
    runs = [b for r in owned for b, _ in r]
    assert all(b % unit == 0 for b in runs)
    if n >= unit * world * 4:
        assert all(3 <= len(r) <= 5 for r in owned)
        # interleaved: consecutive runs belong to consecutive ranks
        order = sorted((b, q) for q, r in enumerate(owned) for b, _ in r)
        assert [q for _, q in order[:world]] == list(range(world))


@pytest.mark.parametrize("world,total,reset_at", [(2, None, -1), (3, 3 * PATHS + 1001, -1), (2, None, 1), (4, 5, -1)])
def test_reduce_two_phase_update_matches_single_process(world, total, reset_at, tmp_path):
    """The reduce exchange with HipEngine's update schedule (radii from the
    all-reduced counts before the next gather, the owner's flux after it,
    so the flux reduce-scatter overlaps a whole pass), over gloo: the same
    records as one process — also across a reset between passes (the reset
    discards the pass whose flux is still in flight) and with ranks that hold
    no paths."""
    mp.start_processes(_worker, args=(world, _free_port(), "reduce", str(tmp_path), total, True, reset_at),
                       nprocs=world, join=True, start_method="spawn")
    ref_recs, ref_img = _single_process_reference(world, total, reset_at)
    idx = np.concatenate([np.load(tmp_path / f"idx{r}.npy") for r in range(world)])
    recs = np.concatenate([np.load(tmp_path / f"recs{r}.npy") for r in range(world)]).view(RECORD_DTYPE)
    assert np.array_equal(np.sort(idx), np.nonzero((ref_recs["flags"] & 7) == 0)[0])
    ref_recs = ref_recs[idx]
    assert np.array_equal(recs["photon_count"], ref_recs["photon_count"])
    assert np.array_equal(recs["radius2"].view(np.uint32), ref_recs["radius2"].view(np.uint32))
    np.testing.assert_allclose(recs["flux"], ref_recs["flux"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(np.load(tmp_path / "img0.npy"), ref_img, rtol=1e-5, atol=1e-6)
