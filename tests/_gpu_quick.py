import sys, time, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import ggnn_oracle as O
import torch
from ggnn_amd.engine import PropagationEngine
def nrms(x, r): return np.sqrt(np.mean((x-r)**2))/np.sqrt(np.mean(r**2))
for prec in ("fp16", "bf16", "fp32"):
  for (b,v,h,C,T) in [(8,64,128,4,3),(2,128,256,8,2),(4,100,256,4,3),(2,128,256,8,5)]:
    A, h0 = O.synthetic_batch(b, v, h, C, seed=b+v)
    w = O.synthetic_weights(h, C, seed=3)
    A64 = A.astype(np.float64); w64 = {k: x.astype(np.float64) for k,x in w.items()}
    hT, caches = O.forward(A64, h0.astype(np.float64), w64, T)
    dhT = np.random.default_rng(1).standard_normal((b,v,h)).astype(np.float32)
    g = O.backward(A64, dhT.astype(np.float64), caches, w64)
    eng = PropagationEngine(h, C, precision=prec)
    dev = eng.device
    pack = eng.pack_weights({k: torch.from_numpy(x).to(dev) for k,x in w.items()})
    eng.set_adjacency(torch.from_numpy(A).to(dev))
    out = eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=True).cpu().numpy()
    gg = eng.backward(torch.from_numpy(dhT).to(dev))
    torch.cuda.synchronize()
    print(prec, (b,v,h,C,T), 'fwd max %.2e nrms %.2e' % (np.abs(out-hT).max(), nrms(out, hT)),
          ' grads nrms max %.2e  nmax max %.2e' % (max(nrms(gg[k].cpu().numpy().reshape(g[k].shape), g[k]) for k in g),
                                                  max(np.abs(gg[k].cpu().numpy().reshape(g[k].shape)-g[k]).max()/np.abs(g[k]).max() for k in g)), flush=True)
