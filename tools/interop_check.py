"""Checks that libpmhip.so and torch share one HIP runtime when torch is imported first,
and prints first C2 stage timings."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
import torch
x = torch.zeros(4, device="cuda")
print("torch ok", torch.cuda.get_device_name(0), flush=True)
from pmrender import hip, scenes
from pmrender.abi import RenderParams, PM_GATHER_KDTREE
ctx = scenes.cornell_box(1920, 1080).load_into(hip.Context(0))
p = RenderParams.defaults()
for i in range(3):
    t = time.time(); img, st = ctx.render(p); dt = time.time() - t
    print(f"render {dt*1e3:.1f} ms", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
part = torch.zeros((ctx.num_records(), 4), device="cuda")
torch.cuda.synchronize()
ctx.gather_partial(p, part.data_ptr())
ctx.synchronize()
print("partial M sum", float(part[:, 0].sum()), flush=True)
pk = RenderParams.defaults(gather_structure=PM_GATHER_KDTREE)
ctx.set_counting(True)
img, st = ctx.render(pk)
print("kd", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
img, st = ctx.render(p)
print("grid", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
print("libs:", [l.split()[-1] for l in open('/proc/self/maps') if 'amdhip' in l][:1], flush=True)
