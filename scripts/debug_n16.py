import sys, numpy as np, torch
sys.path.insert(0, '.')
from tests.golden_io import load_golden
from tests.test_gpu_parity import run_hip
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from oracle.fedavg_oracle import fedavg_flat
dev = torch.device('cuda', 0)
case = load_golden()['n16_f32_float']
for ws in (64, 16, 9, 8, 5, 3):
    res = run_hip(case, dev, ws)
    bad = []
    for k, want in case.expected.items():
        got = res.parameter[k].cpu().numpy()
        d = np.nonzero(got.reshape(-1).view(np.uint64) != want.reshape(-1).view(np.uint64))[0]
        if len(d):
            bad.append((k, len(d), d[:5].tolist(), (got.reshape(-1)[d[:3]] - want.reshape(-1)[d[:3]]).tolist()))
    print('wave', ws, 'mismatch', bad)
# context-level: conv1.weight only, K=16, compare with fedavg_flat
xs = [a.arrays['conv1.weight'].reshape(-1) for a in case.arrivals]
ws = [a.weight for a in case.arrivals]
want = fedavg_flat(xs, ws)
lay = ModelLayout.flat(432)
for K in (16,):
    ctx = FedAvgContext(lay, dev)
    t = ClientTable(1)
    for x, w in zip(xs, ws):
        t.add_client([torch.from_numpy(x.copy()).to(dev)], [w])
    out = [torch.empty(432, dtype=torch.float64, device=dev)]
    ctx.aggregate(t, torch.float32, out, torch.float64)
    got = out[0].cpu().numpy()
    d = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    print('ctx K=16 mismatches', len(d), d[:10])
    # sequential oracle variants
    acc = xs[0].astype(np.float64) * ws[0]
    for x, w in zip(xs[1:], ws[1:]):
        acc = acc + x.astype(np.float64) * w
    tot = 0.0
    for w in ws: tot += w
    alt = acc / tot
    print('tot', repr(tot), repr(sum(ws)))
    d2 = np.nonzero(got.view(np.uint64) != alt.view(np.uint64))[0]
    print('vs alt', len(d2))
    # compare acc * W
    print('got*tot - acc max', np.max(np.abs(got * tot - acc)))
