# A/B: C2 step (zero + build) launched eagerly vs replayed from a captured HIP graph
import sys, time, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "storage-engine_amd"))
import torch, lsmbloom
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
ctx = lsmbloom.Context(0)
n = 100_000_000
nb, k = lsmbloom.params(n, 0.01)
keys = torch.empty((n, 16), dtype=torch.uint8, device=dev)
ctx.gen_key16_dev(0x5EED0001, 0, n, keys)
words = torch.zeros(lsmbloom.num_words(nb), dtype=torch.int64, device=dev)
ctx.set_timing(False)
def step():
    words.zero_()
    ctx.build_fixed_dev(keys, 16, n, nb, k, words)
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    for _ in range(5): step()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    step()
torch.cuda.synchronize()
ref = None
for rep in range(3):
    for mode in ("eager", "graph"):
        torch.cuda.synchronize(); t = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(40):
                if mode == "eager": step()
                else: g.replay()
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 40 * 1e3
        w = words.cpu()
        if ref is None: ref = w.clone()
        print(mode, "%.4f ms/step" % dt, "same words:", bool(torch.equal(ref, w)))
