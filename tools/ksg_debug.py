"""Debug aid for the gemm key switch: where it differs from the lane form."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import tfhe_amd  # noqa: E402

c = tfhe_amd.Context("128", 0)
c.keygen(42, 43)
for B in (600, 1024, 1500):
    lv1 = np.random.default_rng(B).integers(0, 1 << 32, (B, 1025), dtype=np.uint64).astype(np.uint32)
    want = c.key_switch(lv1)
    with c.options(ks_form=2):
        got = c.key_switch(lv1)
        got2 = c.key_switch(lv1)
    bad = got != want
    rows = np.nonzero(bad.any(axis=1))[0]
    cols = np.nonzero(bad.any(axis=0))[0]
    print(B, "bad words", int(bad.sum()), "rows", len(rows), rows[:10], rows[-5:], "cols", len(cols), cols[:10],
          "repeat equal", np.array_equal(got, got2))
