"""The multi-GPU pass runner (pmrender/dist.py) with the real HIP engine:
two ranks share the one GPU of the test box and talk over gloo (RCCL needs
one GPU per rank; the driver's 8-GPU bench uses it). Exercises the
active-record view, the pipelined exchange, pm_final_view and the slot
all-gather on the device, against one context over the same global paths —
both exchanges are bit-exact (exact fixed-point sums, canonical buckets)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu

PATHS, PASSES, W, H = 8192, 3, 64, 48


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, exchange, outdir, backend="gloo", reset_at=-1, fused=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cuda-raytrace_amd")]
    import torch  # noqa: F811  (before libpmhip: one HIP runtime)
    from pmrender import hip, scenes
    from pmrender.abi import RenderParams
    from pmrender.dist import HipEngine, PassRunner
    if backend == "nccl":   # RCCL: one rank per GPU, so world 1 on the test box
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = scenes.cornell_box(W, H).load_into(hip.Context(0))
    p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=25.0)
    with torch.cuda.stream(torch.cuda.Stream()):
        eng = HipEngine(ctx)
        if fused:   # the one-kernel update after both collectives (pm_ppm_update_split)
            eng.ppm_update_radius = None
        ctx.eye_pass(p, eng._s())
        runner = PassRunner(eng, p, rank, world, exchange, force_exchange=True)
        assert runner.multi
        for k in range(PASSES):
            runner.step(k, reset=k == reset_at)
        out = torch.zeros((runner.n_records, 3), dtype=torch.float32, device="cuda")
        runner.final_gather(float(runner.emitted_per_pass * PASSES), out)
        torch.cuda.synchronize()
    np.save(os.path.join(outdir, f"img{rank}.npy"), out.cpu().numpy())
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


def _single_context_image(world, hip_mod, reset_at=-1):
    from pmrender import scenes
    from pmrender.abi import RenderParams
    ref = scenes.cornell_box(W, H).load_into(hip_mod.Context(0))
    p = RenderParams.defaults(paths_per_pass=world * PATHS, initial_radius2=25.0)
    ref.eye_pass(p)
    for k in range(PASSES):
        if k == reset_at:
            ref.reset_records(p)
        ref.trace_photons(p, k, 0, world * PATHS)
        ref.build_photon_map(p)
        ref.gather(p)
    n = ref.num_records()
    img = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ref.final(float(world * PATHS * PASSES), 0, n, img.data_ptr())
    ref.synchronize()
    want = img.cpu().numpy()
    ref.close()
    return want


@pytest.mark.parametrize("exchange", ["reduce", "allgather"])
def test_two_ranks_one_gpu_match_single_context(exchange, tmp_path, hip_mod):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), exchange, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    want = _single_context_image(world, hip_mod)
    for r in range(world):
        got = np.load(tmp_path / f"img{r}.npy")
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"rank {r} image differs"


@pytest.mark.parametrize("exchange", ["reduce", "allgather"])
def test_rccl_world1_exchange_matches_single_context(exchange, tmp_path, hip_mod):
    """The RCCL branch of the exchange (dist.py _AsyncExchange.start: async
    all_reduce + reduce_scatter_tensor on the device tensors, joined by a
    stream-ordered wait; all_gather_into_tensor of the slots) on an nccl
    process group of world size 1, the N > 1 path forced (record view,
    pm_gather_split, pm_ppm_update_split, pm_final_view / bands): image bit
    for bit equal to one context without any exchange."""
    mp.start_processes(_worker, args=(1, _free_port(), exchange, str(tmp_path), "nccl"), nprocs=1, join=True,
                       start_method="spawn")
    want = _single_context_image(1, hip_mod)
    got = np.load(tmp_path / "img0.npy")
    assert (want > 0).any()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"RCCL world-1 {exchange} image differs"


@pytest.mark.parametrize("mode", ["late", "fused"])
def test_two_ranks_reduce_with_reset(mode, tmp_path, hip_mod):
    """The reduce exchange's two update schedules — radii from the counts
    before the next gather and flux after it (the default, so the flux
    reduce-scatter overlaps the next pass's gather), or one fused update after
    both collectives — with a PPM reset between passes (bench.py's per-step
    pattern): images bit for bit equal to one context."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), "reduce", str(tmp_path), "gloo", 1, mode == "fused"),
                       nprocs=world, join=True, start_method="spawn")
    want = _single_context_image(world, hip_mod, reset_at=1)
    for r in range(world):
        got = np.load(tmp_path / f"img{r}.npy")
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"rank {r} image differs ({mode})"
