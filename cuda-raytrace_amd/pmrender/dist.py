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
    40-B photon slots into a replicated map, gather locally owned chunks.
    Bytes per pass: 40 B x slots x (N-1)/N per rank.

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
    def __init__(self, engine, params, rank=0, world=1, exchange="reduce"):
        if exchange not in ("reduce", "allgather"):
            raise ValueError(exchange)
        if world > 1 and exchange == "reduce" and int(getattr(params, "estimator", 0)) != 0:
            # the kNN estimate is not a sum over photon shards
            raise ValueError("the kNN estimator needs the all-gather exchange")
        self.e, self.p, self.rank, self.world, self.exchange = engine, params, rank, world, exchange
        self.paths = int(params.paths_per_pass)           # per rank
        self.path_begin = rank * self.paths
        self.slots_per_rank = self.paths * int(params.max_photon_count)
        n = engine.num_records()
        self.n_records = n
        self.rec_begin, self.rec_count, self.rec_per = _chunk(n, world, rank)   # final image split
        self.padded = self.rec_per * world
        self.slot_buf = None
        self._pending = None
        if world > 1 and exchange == "reduce":
            # exchange over the active records only, owned in contiguous chunks of the view
            self.n_view = engine.set_record_view(True)
            self.v_begin, self.v_count, self.v_per = _chunk(self.n_view, world, rank)
            # per active record: photon count M (int32, all-reduced) and flux L.rgb
            # (int64 fixed point, reduce-scattered); the sums over ranks are exact.
            # Rows past n_view stay zero.
            self.count = engine.alloc((self.v_per * world,), torch.int32)
            self.flux = engine.alloc((self.v_per * world, 3), torch.int64)
            self.flux_chunk = engine.alloc((self.v_per, 3), torch.int64)
        if world > 1 and exchange == "allgather":
            self.slot_buf = engine.alloc((world * self.slots_per_rank * PHOTON_DTYPE.itemsize,), torch.uint8)
            engine.use_slot_buffer(self.slot_buf)

    @property
    def emitted_per_pass(self):
        return self.paths * self.world

    # gloo (CPU tests, or several ranks sharing one GPU) has no reduce_scatter
    # and works on host tensors: device tensors are staged through host memory
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
        if self._gloo():
            self._pending = ("gloo", None)   # done synchronously in _finish_exchange
        else:
            self._pending = ("rccl", [dist.all_reduce(self.count, async_op=True),
                                      dist.reduce_scatter_tensor(self.flux_chunk, self.flux, async_op=True)])

    def _finish_exchange(self):
        """Complete the previous pass: global counts -> every radius; summed flux -> owner's chunk."""
        if self._pending is None:
            return
        kind, works = self._pending
        self._pending = None
        if kind == "gloo":                   # gloo has no reduce_scatter: all-reduce + slice, via host
            for t in (self.count, self.flux):
                host = t.cpu()
                dist.all_reduce(host)
                t.copy_(host)
            self.flux_chunk.copy_(self.flux[self.rank * self.v_per:(self.rank + 1) * self.v_per])
        else:
            for w in works:
                w.wait()                     # the compute stream waits for the collectives
        self.e.ppm_update_split(self.p, self.count, self.flux_chunk, self.v_begin, self.v_count)

    def flush(self):
        """Finish the exchange still in flight (call before reading records or timing)."""
        self._finish_exchange()

    def step(self, pass_index, reset=False):
        """One PPM pass: trace this rank's paths, build, gather (+ exchange)."""
        e, p = self.e, self.p
        if self.world == 1:
            if reset:
                e.reset_records(p)
            e.trace_photons(p, pass_index, 0, self.paths, 0)
            e.build_photon_map(p, self.slots_per_rank)
            e.gather(p)
            return
        if self.exchange == "reduce":
            # trace + build do not read records: they overlap the previous exchange
            e.trace_photons(p, pass_index, self.path_begin, self.paths, self.path_begin)
            e.build_photon_map(p, self.slots_per_rank)
            self._finish_exchange()
            if reset:
                e.reset_records(p)
            e.gather_split(p, self.count, self.flux)
            self._start_exchange()
        else:
            if reset:
                e.reset_records(p)
            e.trace_photons(p, pass_index, self.path_begin, self.paths, 0)
            mine = self.slot_buf[self.rank * self.slots_per_rank * PHOTON_DTYPE.itemsize:
                                 (self.rank + 1) * self.slots_per_rank * PHOTON_DTYPE.itemsize]
            self._all_gather(self.slot_buf, mine)
            e.build_photon_map(p, self.world * self.slots_per_rank)
            e.gather_range(p, self.rec_begin, self.rec_count)   # replicated map, owned records

    def final_gather(self, emitted, out_full):
        """Final radiance of all records (record order) on every rank."""
        self.flush()
        if self.world == 1:
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
        mine = self.e.alloc((self.rec_per, 3), torch.float32)
        self.e.final(emitted, self.rec_begin, self.rec_count, mine)
        gathered = self.e.alloc((self.padded, 3), torch.float32)
        self._all_gather(gathered, mine)
        out_full.copy_(gathered[: self.n_records])
        return out_full
