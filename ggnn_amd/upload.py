"""Host -> device uploads of per-batch feeds through a reused pinned buffer.

``tensor.to(device)`` from pageable numpy memory is synchronous: it waits for
every kernel already queued on the stream, so each of a batch's uploads (edge
lists, word inputs, labels) drained the GPU and serialised host batching with
device work.  An ``Uploader`` copies the array into its own page-locked buffer
and issues an asynchronous copy on the current stream; before the buffer is
reused, it waits for the previous copy (an event), which has normally long
completed.  One uploader per call site, so uploads of one batch never share a
buffer.
"""
from __future__ import annotations

import numpy as np
import torch

_DTYPES = {np.dtype(np.float32): torch.float32, np.dtype(np.int32): torch.int32,
           np.dtype(np.int64): torch.int64, np.dtype(np.float64): torch.float64}


class Uploader:
    def __init__(self):
        self._buf = None
        self._event = None

    def __call__(self, arr, device) -> torch.Tensor:
        arr = np.ascontiguousarray(arr)
        dt = _DTYPES.get(arr.dtype)
        dev = torch.device(device)
        if dt is None or dev.type != "cuda":
            return torch.from_numpy(arr).to(dev)
        n = arr.nbytes
        out = torch.empty(arr.shape, dtype=dt, device=dev)
        if n == 0:
            return out
        if self._event is not None:
            self._event.synchronize()  # the previous upload has left the buffer
        if self._buf is None or self._buf.numel() < n:
            self._buf = torch.empty(max(n, 1 << 16) * 2, dtype=torch.uint8, pin_memory=True)
        host = self._buf[:n]
        host.numpy()[...] = arr.reshape(-1).view(np.uint8)
        out.view(-1).view(torch.uint8).copy_(host, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record(torch.cuda.current_stream(dev))
        return out
