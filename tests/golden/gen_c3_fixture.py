#!/usr/bin/env python3
"""C3 at full size (10 M keys x 8 SST filters): digests of the oracle's answers
for bench.py's probe leg (tests/c3_ref.py has the workload), so the bench line
can say every answer equals the oracle's without running the oracle.

Run here (CPU): python3 tests/golden/gen_c3_fixture.py  (~1 min)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import c3_ref  # noqa: E402
import oracle_ct  # noqa: E402


def main():
    orc = oracle_ct.load()
    Q, F = 10_000_000, 8
    mask, fset, mixed = c3_ref.answers(orc, Q, F, threads=os.cpu_count() or 8)
    out = {"what": "C3: 10 M key16 lookups (first half members, torch.randint seed 1) x 8 filters new(1000, 0.01) "
                   "from key16(0xF000 + f, 0..1000); answers of the CPU oracle",
           "Q": Q, "F": F,
           "probe_mask_sha256": c3_ref.sha(mask.astype(np.uint8)),
           "probe_positive_rows": int((mask != 0).any(axis=1).sum()),
           "fset_mask_sha256": c3_ref.sha(fset.astype("<u8")),
           "fset_nonzero_rows": int((fset != 0).sum()),
           "fset_mixed_mask_sha256": c3_ref.sha(mixed.astype("<u8")),
           "fset_mixed_nonzero_rows": int((mixed != 0).sum())}
    with open(os.path.join(HERE, "c3_fixture.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
