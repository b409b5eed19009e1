import sys, time, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import ggnn_oracle as O
import torch
from ggnn_amd.engine import PropagationEngine
print(torch.cuda.get_device_name(0), flush=True)
for (b,v,h,C,T) in [(3,20,128,4,2),(8,64,128,4,3),(2,128,256,8,2),(4,100,256,4,3)]:
    A, h0 = O.synthetic_batch(b, v, h, C, seed=b+v)
    w = O.synthetic_weights(h, C, seed=3)
    A64 = A.astype(np.float64); w64 = {k: x.astype(np.float64) for k,x in w.items()}
    hT, caches = O.forward(A64, h0.astype(np.float64), w64, T)
    dhT = np.random.default_rng(1).standard_normal((b,v,h)).astype(np.float32)
    g = O.backward(A64, dhT.astype(np.float64), caches, w64)
    eng = PropagationEngine(h, C)
    dev = eng.device
    tw = {k: torch.from_numpy(x).to(dev) for k,x in w.items()}
    pack = eng.pack_weights(tw)
    eng.set_adjacency(torch.from_numpy(A).to(dev))
    out = eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=True)
    gg = eng.backward(torch.from_numpy(dhT).to(dev))
    torch.cuda.synchronize()
    print((b,v,h,C,T), 'fwd maxerr %.3e' % np.abs(out.cpu().numpy()-hT).max(), flush=True)
    for k in ("h0","edge_weights","edge_biases","gates_kernel","gates_bias","candidate_kernel","candidate_bias"):
        r = g[k]; x = gg[k].cpu().numpy().reshape(r.shape)
        print('   %-16s rel %.3e  (refmax %.3e)' % (k, np.abs(x-r).max()/np.abs(r).max(), np.abs(r).max()), flush=True)
