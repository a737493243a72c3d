"""Delivery of the device history into the reference's host arrays.

``WR.core_ray_run_rk45`` fills ``rlon ... rvg`` (``(nt, 3, nsource, nzwn)``
fp64 each, ``wr.py:160-167, 868-876``) row by row.  The GPU path produces
rows in chunks of ``[nray][rows][8]`` (``engine.RayEngine.integrate``);
``HistorySink`` moves each chunk into those arrays while the GPU already
integrates the next one:

  compute stream   launch k ──────────── launch k+1 ─────────── launch k+2
  copy stream        └─ permute(k) → D2H(k) into pinned staging
  host threads                         └─ 7 memcpys into rlon..rvg [i0:i1]

* two device row buffers alternate (``buffers()``); launch k+2 waits for the
  permute of chunk k before it overwrites that buffer;
* the permute to ``[7][rows][nray]`` (the reference layout per variable) runs
  on the device; the D2H goes into page-locked staging (DMA at PCIe rate);
* the host copies run in a thread pool (NumPy releases the GIL for them);
  staging buffer b is reused only after chunk k-2's copies finished.

``finish()`` waits for everything; afterwards the arrays hold exactly the
rows the device produced (tests/test_gpu_parity.py::test_dropin_history_*).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

F64 = torch.float64
_PINNED = {}


def _pinned(shape):
    """Two page-locked staging buffers, kept across runs (pinning is slow)."""
    key = tuple(shape)
    if key not in _PINNED:
        _PINNED.clear()
        _PINNED[key] = [torch.empty(key, dtype=F64, pin_memory=True) for _ in range(2)]
    return _PINNED[key]


class HistorySink:
    def __init__(self, hist, rows_shape, nray, max_rows, device, progress=None, workers=8):
        self.hist, self.rows_shape, self.nray = hist, rows_shape, nray
        self.progress = progress
        self.device = device
        self.copy_stream = torch.cuda.Stream(device=device)
        self.stage_dev = [torch.empty((7, max_rows, nray), dtype=F64, device=device) for _ in range(2)]
        self.stage_host = _pinned((7, max_rows, nray))
        self.out = [torch.empty((nray, max_rows, 8), dtype=F64, device=device) for _ in range(2)]
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.futs = [[], []]
        self.perm_done = [None, None]
        self.k = 0

    def buffers(self):
        """The two device row buffers the engine alternates between."""
        return self.out

    def _copy_rows(self, ev, b, v, i0, i1):
        ev.synchronize()
        r = i1 - i0
        src = self.stage_host[b].numpy()[v, :r]
        self.hist[v][i0:i1] = src.reshape((r,) + self.rows_shape)

    def __call__(self, i0, i1, view):
        k, b = self.k, self.k % 2
        self.k += 1
        r = i1 - i0
        # launch k+1 writes the buffer chunk k-1 was read from
        if self.perm_done[1 - b] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.perm_done[1 - b])
        # staging b was last used by chunk k-2
        for f in self.futs[b]:
            f.result()
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(ready)
            dst = self.stage_dev[b][:, :r]
            dst.copy_(view[:, :, :7].permute(2, 1, 0))
            perm = torch.cuda.Event()
            perm.record(self.copy_stream)
            self.stage_host[b][:, :r].copy_(dst, non_blocking=True)
            d2h = torch.cuda.Event()
            d2h.record(self.copy_stream)
        self.perm_done[b] = perm
        self.futs[b] = [self.pool.submit(self._copy_rows, d2h, b, v, i0, i1) for v in range(7)]
        if self.progress is not None:
            self.progress(i1 - 1)

    def finish(self):
        for fs in self.futs:
            for f in fs:
                f.result()
        self.copy_stream.synchronize()
        self.pool.shutdown(wait=True)
