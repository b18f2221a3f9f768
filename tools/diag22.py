import os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(R, "storage-engine_amd"), os.path.join(R, "tests")]
os.environ["LSMB_SLICE_LOG2"] = "22"
import numpy as np, keygen, lsmbloom, oracle_ct
orc = oracle_ct.load(); ctx = lsmbloom.Context(0)
for n, fk in ((2_000_000, 10**8), (2_000_000, 2 * 10**8), (2_000_000, 10**9)):
    nb, k = lsmbloom.params(fk, 0.01)
    keys = keygen.key16(0x5EED2222, 0, n)
    got = ctx.build_fixed(keys, 16, nb, k); ref = orc.build_fixed_mt(keys, 16, nb, k, 16)
    bad = np.nonzero(got != ref)[0]
    missing = np.bitwise_count(ref[bad] & ~got[bad]).sum(); extra = np.bitwise_count(got[bad] & ~ref[bad]).sum()
    bins = np.unique(bad * 64 >> 22)
    print("n", n, "num_bits", nb, "bins", (nb + (1 << 22) - 1) >> 22, "bad words", bad.size, "missing bits", int(missing), "extra bits", int(extra), "bins", bins.size, bins[:10], "quarters", np.bincount((bad * 64 >> 20) % 4, minlength=4))
    print("  popcount got/ref", int(np.bitwise_count(got).sum()), int(np.bitwise_count(ref).sum()))
