"""One progressive photon pass across N GPUs (one process per GPU).

Work split:
  * photon paths: rank r traces paths [r*P, (r+1)*P) with GLOBAL path ids, so
    the Halton index and the Philox counter of every slot are the same as
    in a 1-GPU run (owner-writes, photontracing.cu:93,144);
  * gather records: every rank holds the full eye-pass record set (the eye
    pass is deterministic and cheap, so it is replicated instead of
    exchanged); PPM state is owned per contiguous chunk of the ACTIVE
    records (pm_set_record_view: MISS / EXCEPTION / padding records never
    take part in the exchange — 47% of the records at C2).

Two exchange strategies:
  * "reduce" (default): each rank builds a map of ITS photons and gathers all
    records against it; the PPM estimator's sums (M, L) are linear in the
    photon set, so summing the per-rank partials (M as int32, the flux as
    three int64 in the gather's exact fixed point) gives the 1-GPU result
    bit for bit. The radius / photon-count update needs only M, so the
    counts are ALL-REDUCED and every rank updates every radius itself (no
    radius exchange); the flux is REDUCE-SCATTERED to the owner of each
    view chunk, which updates its flux. Bytes on xGMI per pass: 4 B
    (all-reduce) + 24 B (reduce-scatter) per active record, independent of
    the photon count. Both collectives are issued asynchronously right after
    the gather and only waited for after the NEXT pass's trace and bucket
    build (which do not read records), so they overlap them; flush()
    completes the last one.
  * "allgather": the reference-style exchange: all-gather the
    40-B photon slots into a replicated map, gather the locally owned records:
    the image's 8-row bands, dealt round-robin in runs (about four per rank)
    so that every rank gets a mix of bright and dark image regions. Bytes per
    pass: 40 B x slots x (N-1)/N per rank.

Records: in "reduce" mode every rank gathers EVERY active record against its
own photons (the gather is replicated, the photon map is not); in
"allgather" mode the map is replicated and the records are split.

The engine protocol (implemented by HipEngine below for the GPU and by the
CPU oracle engine in tests/) works on torch tensors so that the collective
logic is identical for RCCL (GPU) and gloo (CPU tests).
"""
import ctypes

import torch
import torch.distributed as dist

from .abi import PHOTON_DTYPE


def _chunk(n, world, rank):
    per = (n + world - 1) // world
    b = min(n, rank * per)
    return b, min(n, b + per) - b, per


def _bands(n, unit, world, per_rank=4):
    """Record ranges of each rank in the all-gather mode: the image's 8-row
    bands (`unit` records each) in runs of equal size dealt round-robin, about
    `per_rank` runs per rank — Cornell photon density is non-uniform over the
    image, interleaving balances the gather."""
    units = (n + unit - 1) // unit
    runs = max(1, -(-units // (world * per_rank)))      # bands per run
    owned = [[] for _ in range(world)]
    k = 0
    for u in range(0, units, runs):
        b = u * unit
        owned[k % world].append((b, min(n, (u + runs) * unit) - b))
        k += 1
    return owned


class _AsyncExchange:
    """The reduce exchange of one pass, one contract for every backend:
    start() issues the count all-reduce and the flux reduce-scatter
    asynchronously, wait() joins them — afterwards `count` holds the global
    photon counts of every view record and `flux_chunk` this rank's slice of
    the summed flux; wait_count() joins the count all-reduce alone (the radii
    need it before the next gather, the flux only after it). The backend enters in one place: RCCL runs
    reduce_scatter_tensor on the device tensors; gloo (the CPU tests, and
    several ranks sharing one GPU) has no reduce-scatter, so it all-reduces
    the flux (on host copies for device tensors) and slices at wait()."""

    def __init__(self, count, flux, flux_chunk, rank, v_per):
        self.count, self.flux, self.flux_chunk = count, flux, flux_chunk
        self.rank, self.v_per = rank, v_per
        self.gloo = dist.get_backend() == "gloo"
        self.works = []
        self.host = None

    def start(self):
        if not self.gloo:
            self.works = [dist.all_reduce(self.count, async_op=True),
                          dist.reduce_scatter_tensor(self.flux_chunk, self.flux, async_op=True)]
            return self
        count, flux = self.count, self.flux
        if count.is_cuda:                      # gloo works on host tensors
            count, flux = count.cpu(), flux.cpu()
            self.host = (count, flux)
        self.works = [dist.all_reduce(count, async_op=True), dist.all_reduce(flux, async_op=True)]
        return self

    def wait_count(self):
        """the count all-reduce only (the flux reduce-scatter may continue)"""
        if self.works[0] is not None:
            self.works[0].wait()               # RCCL: the compute stream waits for the collective
            self.works[0] = None
            if self.gloo and self.host is not None:
                self.count.copy_(self.host[0])

    def wait(self):
        self.wait_count()
        if self.works[1] is not None:
            self.works[1].wait()
            self.works[1] = None
            if self.gloo:
                flux = self.host[1] if self.host is not None else self.flux
                self.flux_chunk.copy_(flux[self.rank * self.v_per:(self.rank + 1) * self.v_per])


class HipEngine:
    """Adapter of hip.Context onto torch tensors; all stages run on torch's
    current stream so they are ordered with the RCCL collectives."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.device = torch.device("cuda", torch.cuda.current_device())

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def num_records(self):
        return self.ctx.num_records()

    def band_records(self):
        """Records of one 8-pixel-row band: records are stored in 8x8 tiles
        (one wave each), so a tile row is a contiguous record range."""
        if self.ctx.pinhole:
            return ((self.ctx.width + 7) // 8) * 64
        return 8 * 64

    def alloc(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype, device=self.device)

    def use_slot_buffer(self, t):
        self.ctx.set_slot_buffer(t.data_ptr(), t.numel() // PHOTON_DTYPE.itemsize)

    def reset_records(self, p):
        self.ctx.reset_records(p, self._s())

    def set_record_view(self, active_only=True):
        return self.ctx.set_record_view(active_only)

    def trace_photons(self, p, pass_index, path_begin, path_count, slot_path_base):
        self.ctx.trace_photons(p, pass_index, path_begin, path_count, slot_path_base, self._s())

    def build_photon_map(self, p, n_slots):
        self.ctx.build_photon_map(p, n_slots, self._s())

    def gather(self, p):
        self.ctx.gather(p, self._s())

    def gather_range(self, p, rec_begin, rec_count):
        self.ctx.gather_range(p, rec_begin, rec_count, self._s())

    def gather_partial(self, p, out):
        self.ctx.gather_partial(p, out.data_ptr(), self._s())

    def gather_split(self, p, count, flux):
        self.ctx.gather_split(p, count.data_ptr(), flux.data_ptr(), self._s())

    def ppm_update_split(self, p, count, flux_chunk, v_begin, v_count):
        self.ctx.ppm_update_split(p, count.data_ptr(), flux_chunk.data_ptr(), v_begin, v_count, self._s())

    def ppm_update_radius(self, p, count, ratio):
        self.ctx.ppm_update_split_radius(p, count.data_ptr(), ratio.data_ptr(), self._s())

    def ppm_update_flux(self, p, ratio, flux_chunk, v_begin, v_count):
        self.ctx.ppm_update_split_flux(p, ratio.data_ptr(), flux_chunk.data_ptr(), v_begin, v_count, self._s())

    def ppm_update(self, p, partial, rec_begin, rec_count):
        self.ctx.ppm_update(p, partial.data_ptr(), rec_begin, rec_count, self._s())

    def get_radius2(self, rec_begin, rec_count, out):
        self.ctx.get_radius2(rec_begin, rec_count, out.data_ptr(), self._s())

    def set_radius2(self, src, rec_begin, rec_count):
        self.ctx.set_radius2(src.data_ptr(), rec_begin, rec_count, self._s())

    def final(self, emitted, rec_begin, rec_count, out):
        self.ctx.final(emitted, rec_begin, rec_count, out.data_ptr(), self._s())

    def final_view(self, emitted, v_begin, v_count, out):
        self.ctx.final_view(emitted, v_begin, v_count, out.data_ptr(), self._s())

    def record_view_list(self, out):
        self.ctx.record_view_list(out.data_ptr(), self._s())


class PassRunner:
    def __init__(self, engine, params, rank=0, world=1, exchange="reduce", force_exchange=False, total_paths=None):
        """force_exchange: run the N > 1 code path (record view, collectives,
        owned chunks / bands) even at world size 1 — how a 1-GPU box executes
        the RCCL branch of the exchange (tests/test_dist_gpu.py).
        total_paths: strong scaling — the pass emits total_paths paths over
        all ranks (rank r traces global paths [r*per, min(total, (r+1)*per)),
        per = ceil(total / world); the last rank's short chunk leaves its
        tail slots invalid); None: weak scaling, params.paths_per_pass per
        rank."""
        if exchange not in ("reduce", "allgather"):
            raise ValueError(exchange)
        self.multi = world > 1 or force_exchange
        if self.multi and exchange == "reduce" and int(getattr(params, "estimator", 0)) != 0:
            # the kNN estimate is not a sum over photon shards
            raise ValueError("the kNN estimator needs the all-gather exchange")
        self.e, self.p, self.rank, self.world, self.exchange = engine, params, rank, world, exchange
        if total_paths is None:
            self.per = int(params.paths_per_pass)         # chunk per rank
            self.total = self.per * world
        else:
            self.total = int(total_paths)
            self.per = -(-self.total // world)
        self.path_begin = min(self.total, rank * self.per)
        self.paths = min(self.total, self.path_begin + self.per) - self.path_begin   # this rank's paths
        self.slots_per_rank = self.per * int(params.max_photon_count)             # slot chunk per rank
        self.slots_mine = self.paths * int(params.max_photon_count)
        # exchange timing (bench.py, after its timed region): run each exchange
        # to completion at once and record its GPU time (ms) per pass
        self.time_exchange = False
        self.exchange_ms = []
        n = engine.num_records()
        self.n_records = n
        self.rec_begin, self.rec_count, self.rec_per = _chunk(n, world, rank)   # final image split
        self.padded = self.rec_per * world
        self.slot_buf = None
        self._pending = None
        self._radius_done = False
        # pass pipelining (one GPU, HipEngine): the next pass's trace runs on a
        # second stream while this pass gathers (set by the caller, step(next_pass=))
        self.pipeline = False
        self._ahead = None             # (pass, event) of a trace issued ahead
        self._tstream = None
        if self.multi and exchange == "reduce":
            # exchange over the active records only, owned in contiguous chunks of the view
            self.n_view = engine.set_record_view(True)
            self.v_begin, self.v_count, self.v_per = _chunk(self.n_view, world, rank)
            # per active record: photon count M (int32, all-reduced) and flux L.rgb
            # (int64 fixed point, reduce-scattered); the sums over ranks are exact.
            # Rows past n_view stay zero.
            self.count = engine.alloc((self.v_per * world,), torch.int32)
            self.flux = engine.alloc((self.v_per * world, 3), torch.int64)
            self.flux_chunk = engine.alloc((self.v_per, 3), torch.int64)
            # engines with the two-phase update (HipEngine): the radii are
            # updated as soon as the counts have landed, the flux only after the
            # next pass's gather, so the flux reduce-scatter overlaps trace,
            # build AND gather; the gather writes the other of two flux buffers
            self.late_flux = callable(getattr(engine, "ppm_update_radius", None))
            if self.late_flux:
                self.flux_bufs = [self.flux, engine.alloc((self.v_per * world, 3), torch.int64)]
                self.ratio = engine.alloc((self.v_per * world,), torch.float32)
        if self.multi and exchange == "allgather":
            self.slot_buf = engine.alloc((world * self.slots_per_rank * PHOTON_DTYPE.itemsize,), torch.uint8)
            engine.use_slot_buffer(self.slot_buf)
            unit = engine.band_records() if hasattr(engine, "band_records") else 512
            self.bands = _bands(n, unit, world)            # interleaved 8-row bands per rank
            self.band_max = max(sum(c for _, c in b) for b in self.bands)

    @property
    def emitted_per_pass(self):
        return self.total

    def _timed(self, fn):
        """fn() with its GPU time appended to exchange_ms when time_exchange
        is set (CUDA events on the current stream; the collectives are joined
        inside fn, so the stream waits for them before the end event)"""
        if not self.time_exchange or not torch.cuda.is_available():
            return fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r = fn()
        b.record()
        b.synchronize()
        self.exchange_ms.append(a.elapsed_time(b))
        return r

    # gloo (CPU tests, or several ranks sharing one GPU) works on host tensors:
    # device tensors are staged through host memory
    @staticmethod
    def _gloo():
        return dist.get_backend() == "gloo"

    def _all_gather(self, out, mine):
        if self._gloo() and out.is_cuda:
            host = out.cpu()
            dist.all_gather_into_tensor(host, mine.cpu())
            out.copy_(host)
        else:
            dist.all_gather_into_tensor(out, mine)

    def _start_exchange(self):
        self._pending = _AsyncExchange(self.count, self.flux, self.flux_chunk, self.rank, self.v_per).start()
        self._radius_done = False

    def _finish_radius(self):
        """Two-phase update, first half: global counts -> every radius (before the next gather)."""
        if self._pending is None or self._radius_done:
            return
        self._pending.wait_count()
        self.e.ppm_update_radius(self.p, self.count, self.ratio)
        self._radius_done = True

    def _finish_exchange(self):
        """Complete the previous pass: global counts -> every radius; summed flux -> owner's chunk."""
        if self._pending is None:
            return
        if self.late_flux:
            self._finish_radius()
            self._pending.wait()
            self._pending = None
            self.e.ppm_update_flux(self.p, self.ratio, self.flux_chunk, self.v_begin, self.v_count)
            return
        self._pending.wait()
        self._pending = None
        self.e.ppm_update_split(self.p, self.count, self.flux_chunk, self.v_begin, self.v_count)

    def flush(self):
        """Finish the exchange still in flight (call before reading records or
        timing); a trace issued ahead for a pass that will not run is joined.
        The records are those of the passes that ran; the photon slot buffer
        (pm_download_slots) and the fused bucket counts, however, then hold
        the abandoned pass's photons — the next step traces its own pass
        again, but a caller that reads the slots after flush() reads those."""
        self._finish_exchange()
        if self._ahead is not None:
            torch.cuda.current_stream().wait_event(self._ahead[1])
            self._ahead = None

    def step(self, pass_index, reset=False, next_pass=None):
        """One PPM pass: trace this rank's paths, build, gather (+ exchange).
        With self.pipeline (one GPU), next_pass = the pass the caller runs next:
        its trace is issued here, on a second stream, between this pass's build
        and gather."""
        e, p = self.e, self.p
        if not self.multi:
            if self.pipeline:
                self._step_pipelined(pass_index, reset, next_pass)
                return
            if reset:
                e.reset_records(p)
            e.trace_photons(p, pass_index, 0, self.paths, 0)
            e.build_photon_map(p, self.slots_mine)
            e.gather(p)
            return
        if self.exchange == "reduce":
            # trace + build do not read records: they overlap the previous exchange
            if self.paths:
                e.trace_photons(p, pass_index, self.path_begin, self.paths, self.path_begin)
                e.build_photon_map(p, self.slots_mine)
            if self.late_flux:
                # the previous pass's radii before this gather (before a reset,
                # which the next radius update consumes), its flux after it
                self._finish_radius()
                if reset:
                    e.reset_records(p)
                if self._pending is not None and self.flux is self._pending.flux:
                    self.flux = self.flux_bufs[1] if self.flux is self.flux_bufs[0] else self.flux_bufs[0]
            else:
                self._finish_exchange()
                if reset:
                    e.reset_records(p)              # deferred: the split update below consumes it
            if self.paths:
                e.gather_split(p, self.count, self.flux)
            else:
                # strong scaling with more ranks than chunks: no photons here, so
                # this rank adds nothing to the sums (and builds no map, which
                # would otherwise come from stale slots of an earlier pass)
                self.count.zero_()
                self.flux.zero_()
            if self.late_flux:
                self._finish_exchange()             # the previous pass's flux (its reduce-scatter ran meanwhile)
            self._start_exchange()
            if self.time_exchange:
                self._timed(self._finish_exchange)
        else:
            if reset:
                e.reset_records(p)
            if self.paths:
                e.trace_photons(p, pass_index, self.path_begin, self.paths, 0)
            mine = self.slot_buf[self.rank * self.slots_per_rank * PHOTON_DTYPE.itemsize:
                                 (self.rank + 1) * self.slots_per_rank * PHOTON_DTYPE.itemsize]
            self._timed(lambda: self._all_gather(self.slot_buf, mine))
            e.build_photon_map(p, self.world * self.slots_per_rank)
            for b, c in self.bands[self.rank]:                  # replicated map, owned bands
                e.gather_range(p, b, c)

    def _step_pipelined(self, k, reset, next_pass):
        """Pass k with the trace of pass next_pass overlapping its gather.
        The trace writes the slots, the bucket keys / ranks and the cell
        counts; the build reads them (and leaves the counts cleared) and the
        gather reads only the built buckets and the records. So trace(k + 1)
        may start once build(k) is done — on its own stream, concurrent with
        gather(k) — and build(k + 1) follows gather(k) on the main stream. The
        next pass's grid is chosen when its trace is issued, from the radii
        binned by pass k - 1's gather (the grid sets only the cost)."""
        e, p = self.e, self.p
        main = torch.cuda.current_stream()
        if self._ahead is not None and self._ahead[0] == k:
            main.wait_event(self._ahead[1])
        else:
            if self._ahead is not None:          # a trace issued for another pass: let it land first
                main.wait_event(self._ahead[1])
            e.trace_photons(p, k, 0, self.paths, 0)
        self._ahead = None
        if reset:
            e.reset_records(p)
        e.build_photon_map(p, self.slots_mine)
        if next_pass is not None:
            if self._tstream is None:
                self._tstream = torch.cuda.Stream()
            built = torch.cuda.Event()
            built.record(main)
            self._tstream.wait_event(built)
            with torch.cuda.stream(self._tstream):
                e.trace_photons(p, next_pass, 0, self.paths, 0)
                traced = torch.cuda.Event()
                traced.record(self._tstream)
            self._ahead = (next_pass, traced)
        e.gather(p)

    def final_gather(self, emitted, out_full):
        """Final radiance of all records (record order) on every rank."""
        self.flush()
        if not self.multi:
            self.e.final(emitted, 0, self.n_records, out_full)
            return out_full
        if self.exchange == "reduce":
            # owners hold the PPM state of their view chunk; records outside the
            # active view (MISS / EXCEPTION / padding) are black
            mine = self.e.alloc((self.v_per, 3), torch.float32)
            self.e.final_view(emitted, self.v_begin, self.v_count, mine)
            gathered = self.e.alloc((self.v_per * self.world, 3), torch.float32)
            self._all_gather(gathered, mine)
            view = self.e.alloc((self.n_view,), torch.int32)
            self.e.record_view_list(view)
            out_full.zero_()
            out_full[view.long()] = gathered[: self.n_view]
            return out_full
        # all-gather: each rank renders its bands; equal-size (padded) buffers
        # are all-gathered and every rank scatters them back to record order
        mine = self.e.alloc((self.band_max, 3), torch.float32)
        o = 0
        for b, c in self.bands[self.rank]:
            self.e.final(emitted, b, c, mine[o:o + c])
            o += c
        gathered = self.e.alloc((self.band_max * self.world, 3), torch.float32)
        self._all_gather(gathered, mine)
        for q in range(self.world):
            o = q * self.band_max
            for b, c in self.bands[q]:
                out_full[b:b + c] = gathered[o:o + c]
                o += c
        return out_full
