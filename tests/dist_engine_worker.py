"""One rank of the data-parallel training step of the HIP engine, for
tests/test_gpu_dist.py (started as a child process per rank; gloo over the
one GPU of the test box, which is what the 8-GPU RCCL run does per GPU).

Each rank: stage ITS half of the batch, T-step forward + backward through
libggnn.so into a FlatGradients buffer, ONE all-reduce, then ClipAdam with
grad_scale = 1/world (the reference's loss is a per-batch mean,
chem_tensorflow.py:360,399-403).  Rank 0 then repeats the same two steps on the
full batch in one process and writes both results to argv[1] (.npz).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    out = sys.argv[1]
    b, v, h, C, T = (int(x) for x in sys.argv[2].split(","))
    import torch
    import torch.distributed as tdist
    import ggnn_oracle as O
    from ggnn_amd.dist import GRAD_ORDER, FlatGradients, init_from_env
    from ggnn_amd.engine import PropagationEngine
    from ggnn_amd.optim import ClipAdam

    rank, world, _ = init_from_env("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    A, h0 = O.synthetic_batch(b, v, h, C, seed=21)
    w = O.synthetic_weights(h, C, seed=21)
    rng = np.random.default_rng(22)
    dhT = [(rng.standard_normal((b, v, h)) * 2.0 ** -8).astype(np.float32) for _ in range(2)]
    eps = 1e-8  # the reference's Adam epsilon (chem_tensorflow.py:494)

    def dev_t(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)

    def run(sl, reduce):
        """Two training steps on graphs `sl`; returns (params, per-step gradients)."""
        eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision="fp32")
        params = [dev_t(w[k]) for k in GRAD_ORDER]
        wd = dict(zip(GRAD_ORDER, params))
        opt = ClipAdam(params, learning_rate=0.003, epsilon=eps, clamp_gradient_norm=1.0)
        grads = FlatGradients(h, C, True, device=dev)
        gv = dict(grads.views)
        nb = sl.stop - sl.start
        gv["h0"] = torch.empty((nb, v, h), dtype=torch.float32, device=dev)
        eng.set_adjacency(dev_t(A[sl]))
        seen = []
        for it in range(2):
            pack = eng.pack_weights(wd, T=T)
            eng.forward(dev_t(h0[sl]), pack, T, training=True)
            eng.backward(dev_t(dhT[it][sl]), gv)
            if reduce:   # data-parallel: sum over ranks
                grads.all_reduce()
            seen.append(grads.flat.cpu().numpy().copy())
            opt.step([grads.views[k] for k in GRAD_ORDER], grad_scale=1.0 / world)
        torch.cuda.synchronize()
        return np.concatenate([p.detach().cpu().numpy().ravel() for p in params]), np.stack(seen)

    per = b // world
    dp_params, dp_grads = run(slice(rank * per, (rank + 1) * per), True)
    if rank == 0:
        full_params, full_grads = run(slice(0, b), False)
        np.savez(out, dp_params=dp_params, full_params=full_params, dp_grads=dp_grads, full_grads=full_grads,
                 init=np.concatenate([w[k].ravel() for k in GRAD_ORDER]))
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
