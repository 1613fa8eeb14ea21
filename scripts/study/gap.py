# inter-launch gap study on the C2 bench step: events per step / bracket only / hip graph replay
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "dune-hdd_amd", "python"))
import hdd_amd as H
g = H.Grid.structured(H.SIMPLEX, 3200, 640, (0, 0), (5, 1))
loc = g.local()
perm = 10.0 ** np.random.default_rng(10).uniform(-3, 3, 2000)
k = torch.from_numpy(loc.checkerboard((0, 0), (5, 1), 100, 20, perm)).cuda()
ctx = H.Context(0); dm = H.DeviceMesh(loc); dp = H.DevicePattern(loc)
kap = [H.scalar_fn(H.FN_CONST, 1.0)]; ten = H.tensor_fn(H.TENSOR_ISO_PER_ELEM, per_elem=k)
vals = [torch.empty(dp.nnz, dtype=torch.float64, device="cuda")]
fn = lambda: H.assemble(ctx, dm, dp, kap, ten, vals=vals)
K = 20
for _ in range(5): fn()
torch.cuda.synchronize()
def bracket(run):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(); run(); e[1].record(); torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / K
def per_step():
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for a, b in ev:
        a.record(); fn(); b.record()
    return ev
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
gr = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    fn(); torch.cuda.synchronize()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(K): fn()
torch.cuda.synchronize()
for r in range(4):
    a = bracket(lambda: [fn() for _ in range(K)])
    evs = []
    b = bracket(lambda: evs.append(per_step()))
    kin = np.mean([x.elapsed_time(y) for x, y in evs[0]])
    c = bracket(lambda: gr.replay())
    print("round %d: plain %.4f ms/step  events/step %.4f (kernel %.4f)  graph %.4f" % (r, a, b, kin, c), flush=True)
