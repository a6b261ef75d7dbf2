"""Development aid: host time spent inside each gate_batch_dev call (an async call
should return in microseconds; a call that blocks shows the GPU step time)."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, "zig-tfhe_amd")
import tfhe_amd

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
ctx = tfhe_amd.Context("128", device=0)
sk, _ = ctx.keygen(secret_seed=42, cloud_seed=43)
g = np.random.default_rng(1)
A = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=1)
Bc = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=2)
dev = torch.device("cuda", 0)
t_ops = torch.zeros(B, dtype=torch.uint8, device=dev)
t_a = torch.from_numpy(A.view(np.int32)).to(dev)
t_b = torch.from_numpy(Bc.view(np.int32)).to(dev)
t_o = torch.zeros_like(t_a)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
for _ in range(3):
    ctx.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), B)
torch.cuda.synchronize(dev)
calls = []
t0 = time.perf_counter()
for _ in range(10):
    c0 = time.perf_counter()
    ctx.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), B)
    calls.append((time.perf_counter() - c0) * 1e3)
torch.cuda.synchronize(dev)
el = (time.perf_counter() - t0) * 1e3
print(f"B={B}: {el / 10:.3f} ms per step wall; host ms inside each call: " + " ".join(f"{x:.2f}" for x in calls))
