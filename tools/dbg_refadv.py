"""Debug: reference advection solver over the facade vs the device program."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_ref_advection as T  # noqa: E402
import dccrg_amd as D  # noqa: E402

n, M, steps, adapt = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
out = os.path.join(tempfile.mkdtemp(), "r.bin")
ref = T.reference_run(n, M, steps, adapt, out)
dev = T.device_run(n, M, steps, adapt)
m = D.Mapping((n, n, 1), M)
for (s0, dt0, i0, r0), (s1, dt1, i1, r1) in zip(ref, dev):
    a, b = set(i0.tolist()), set(i1.tolist())
    print(f"step {s0}: ref {len(a)} dev {len(b)} only_ref {len(a - b)} only_dev {len(b - a)} dt {dt0!r} {dt1!r}")
    for c in sorted(a - b)[:8]:
        print("  only ref", c, "lvl", m.get_refinement_level(c), "idx", m.get_indices(c))
    for c in sorted(b - a)[:8]:
        print("  only dev", c, "lvl", m.get_refinement_level(c), "idx", m.get_indices(c))
    if a == b:
        d = np.abs(r0 - r1).max()
        print(f"  max |drho| {d:.3e}")
