"""Host overhead of one C4 bench step (development tool): wall time of
pairs_device against the kernel span it reports, and of the pieces around it."""
import sys, time, types
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import torch
import bench
import stem_kernel_amd as ska

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"])
a = types.SimpleNamespace(n=cfg["n"], length=cfg.get("L", 200))
_, ds = bench.build_inputs(cfg, a)
stream = torch.cuda.current_stream(torch.device("cuda", 0))
ctx = ska.Context(0, stream=stream.cuda_stream) if "torchstream" in sys.argv else ska.Context(0)
ctx.upload(ds)
import ctypes
uid = ctypes.create_string_buffer(128)
ska.lib().sk_comm_unique_id(uid, 128)
ctx.comm_init(uid.raw, 0, 1)
kern = bench.make_kernel(cfg["kernel"])
iu, ju = np.triu_indices(a.n)
iu, ju = iu.astype(np.int32), ju.astype(np.int32)
S = cfg["slices"]
per = iu.size // S + 1
out = torch.zeros(per, dtype=torch.float64, device="cuda:0")
gathered = torch.zeros(per, dtype=torch.float64, device="cuda:0")
for rep in range(6):
    t0 = time.perf_counter()
    x, y = iu[rep % S::S], ju[rep % S::S]
    t1 = time.perf_counter()
    ctx.pairs_device(ds, kern, x, y, out.data_ptr())
    t2 = time.perf_counter()
    tm = ctx.last_timing()
    ctx.allgather(out.data_ptr(), per, gathered.data_ptr())
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"allgather call {1e3*(t3-t2):.2f} ms sync {1e3*(t4-t3):.2f} ms", end="  ")
    print(f"slice {1e3*(t1-t0):.2f} ms  pairs_device {1e3*(t2-t1):.2f} ms  kernel span "
          f"{tm['stem_ms']:.2f} ms  host {1e3*(t2-t1)-tm['stem_ms']:.2f} ms", flush=True)
