"""Times the key-switch kernel for B=1024 (128-bit) via the stage API; run under
rocprofv3 --kernel-trace --stats with TFHE_KS_G set."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import numpy as np
import tfhe_amd
pname = sys.argv[1] if len(sys.argv) > 1 else "128"
c = tfhe_amd.Context(pname, 0)
c.keygen(42, 43)
lv1 = np.random.default_rng(0).integers(0, 1 << 32, (1024, 1025), dtype=np.uint64).astype(np.uint32)
ref = c.key_switch(lv1)
for _ in range(4):
    assert np.array_equal(c.key_switch(lv1), ref)
print("ok", os.environ.get("TFHE_KS_G"))
