"""Pass pipelining (pmrender/dist.py PassRunner.pipeline, bench.py
--pipeline): the next pass's trace on a second stream, overlapping this
pass's gather. The records after every schedule must equal the passes run
one after another bit for bit — progressive renders (radii shrink, the
radius histogram sizes later grids), a reset every pass (bench.py's
non-progressive steps), and a schedule whose trace issued ahead is never
used (flush)."""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cuda-raytrace_amd")]


def _run(scene_fn, paths, passes, pipeline, reset_every, r2, drop_last=False, hint=None):
    from pmrender import hip
    from pmrender.abi import RenderParams
    from pmrender.dist import HipEngine, PassRunner
    ctx = scene_fn().load_into(hip.Context(0))
    p = RenderParams.defaults(paths_per_pass=paths, initial_radius2=r2)
    with torch.cuda.stream(torch.cuda.Stream()):
        eng = HipEngine(ctx)
        ctx.eye_pass(p, eng._s())
        runner = PassRunner(eng, p)
        runner.pipeline = pipeline
        for k in range(passes):
            k_pass = 0 if reset_every else k
            nxt = None if k == passes - 1 and not drop_last else (0 if reset_every else k + 1)
            if hint is not None:
                nxt = hint(k)
            runner.step(k_pass, reset=reset_every or k == 0, next_pass=nxt)
        runner.flush()
        torch.cuda.synchronize()
    recs = ctx.download_records()
    ctx.close()
    return recs


def _same(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("scene", ["cornell", "caustic"])
def test_pipelined_progressive_equals_sequential(scene):
    from pmrender import scenes
    fn = (lambda: scenes.cornell_box(96, 64)) if scene == "cornell" else (lambda: scenes.caustic_scene(96, 64))
    seq = _run(fn, 16384, 5, False, False, 16.0)
    pip = _run(fn, 16384, 5, True, False, 16.0)
    _same(seq, pip)


def test_pipelined_reset_every_pass_equals_sequential():
    from pmrender import scenes
    fn = lambda: scenes.cornell_box(96, 64)  # noqa: E731
    seq = _run(fn, 16384, 4, False, True, 16.0)
    pip = _run(fn, 16384, 4, True, True, 16.0)
    _same(seq, pip)


def test_pipelined_unused_trace_ahead_is_joined():
    """the last pass issues a trace ahead that never runs a pass: flush joins
    it, and the records are the passes' that did run"""
    from pmrender import scenes
    fn = lambda: scenes.cornell_box(96, 64)  # noqa: E731
    seq = _run(fn, 16384, 3, False, False, 16.0)
    pip = _run(fn, 16384, 3, True, False, 16.0, drop_last=True)
    _same(seq, pip)


def test_pipelined_mismatched_trace_ahead_is_redone():
    """traces issued ahead for passes that do not come next (the caller's
    next_pass hint is wrong on every other pass): the mismatched trace lands
    first, the pass traces its own photons again (and re-zeroes the fused
    cell counts), so the records equal the sequential passes bit for bit"""
    from pmrender import scenes
    fn = lambda: scenes.cornell_box(96, 64)  # noqa: E731
    seq = _run(fn, 16384, 4, False, False, 16.0)
    pip = _run(fn, 16384, 4, True, False, 16.0, hint=lambda k: k + 1 if k % 2 else k + 3)
    _same(seq, pip)


def test_pipelined_c5_full_size_equals_sequential():
    """bench.py runs C5 (progressive, 1,048,576 paths per pass at 1080p)
    pipelined by default: three full-size passes, records bit for bit."""
    from pmrender import scenes
    fn = lambda: scenes.caustic_scene(1920, 1080)  # noqa: E731
    seq = _run(fn, 1_048_576, 3, False, False, 4.0)
    pip = _run(fn, 1_048_576, 3, True, False, 4.0)
    _same(seq, pip)
