"""Delivery of the device history into the reference's host arrays.

``WR.core_ray_run_rk45`` fills ``rlon ... rvg`` (``(nt, 3, nsource, nzwn)``
fp64 each, ``wr.py:160-167, 868-876``) row by row.  The GPU path produces
rows in chunks of ``[nray][rows][8]`` (``engine.RayEngine.integrate``);
``HistorySink`` moves each chunk into those arrays while the GPU already
integrates the next one, and ships over PCIe only the rays whose rows
changed:

  compute stream  launch k ───────────── launch k+1 ──────────── launch k+2
  copy stream       └ compare(k)  ┌ gather(k) → D2H(k) into pinned staging
  host threads                    │            └ rwrt_host_fill_rows(k)
  main thread     (after launch k+1 is queued) ┘ nonzero(changed k)

* ``compare(k)``: a ray is *changed* in chunk k when any of its 7 delivered
  values in any row differs, bit for bit, from its previous row (kept on the
  device, starting from the host's row 0).  Frozen rays (``rkf45.py:400-403``:
  dead root slots, rays masked earlier -- 70 % of C3's slots) repeat their
  last row forever, so after the first chunk they are never shipped;
* ``gather(k)``: the changed rays' rows, permuted on the device to the
  reference layout ``[7][rows][nchanged]``, then one D2H into page-locked
  staging;
* ``rwrt_host_fill_rows`` (C ABI, host code, GIL released) writes each row
  block of each variable: every column a copy of the previous row (shipped
  with the chunk, 7 x nray doubles, so no chunk's host work waits for
  another's), the shipped columns scattered in -- exactly what copying the
  whole chunk would write;
* two device row buffers alternate (``buffers()``): launch k+2 waits for
  ``gather(k)`` before it overwrites buffer k % 2.

``finish()`` waits for everything; afterwards the arrays hold exactly the
rows the device produced (tests/test_gpu_parity.py::test_dropin_history_*).
"""
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

import _hip as H

F64 = torch.float64
_PINNED = {}            # n -> free pairs of page-locked staging buffers
_PINNED_LOCK = threading.Lock()


def _pinned_take(n):
    """Two page-locked staging buffers of ``n`` doubles for ONE sink: checked
    out of a free list (pinning is slow, so released pairs are reused by the
    next run), never shared by two live sinks -- two runs in two threads (two
    GPUs, two contexts) would otherwise overwrite each other's D2H data."""
    with _PINNED_LOCK:
        free = _PINNED.get(n)
        if free:
            return free.pop()
        if sum(len(v) for v in _PINNED.values()) > 2:
            _PINNED.clear()    # keep at most a few idle pairs pinned
    return [torch.empty(n, dtype=F64, pin_memory=True) for _ in range(2)]


def _pinned_release(n, pair):
    with _PINNED_LOCK:
        _PINNED.setdefault(n, []).append(pair)


def fill_rows(dst, prev, src, cols):
    """``dst[r, ncol]`` (a C-contiguous host block) := ``prev`` in every column
    except ``cols`` (ascending int64), which take ``src[r, len(cols)]``."""
    r, ncol = dst.shape
    n = 0 if cols is None else len(cols)
    H.check(H.load().rwrt_host_fill_rows(
        dst.ctypes.data, r, ncol, dst.strides[0] // 8,
        None if prev is None else prev.ctypes.data,
        None if n == 0 else src.ctypes.data, n, src.strides[0] // 8 if n else 0,
        None if n == 0 else cols.ctypes.data))


class HistorySink:
    def __init__(self, hist, rows_shape, nray, max_rows, device, progress=None, workers=16):
        if not all(h.flags.c_contiguous and h.dtype == np.float64 for h in hist):
            raise ValueError("the history arrays must be C-contiguous float64 (wr.py:160-167)")
        self.hist, self.rows_shape, self.nray = hist, rows_shape, nray
        self.progress = progress
        self.device = device
        self.workers = workers
        self.copy_stream = torch.cuda.Stream(device=device)
        self.stage_dev = [torch.empty(7 * max_rows * nray, dtype=F64, device=device) for _ in range(2)]
        self.stage_n = 7 * max_rows * nray
        self.stage_host = _pinned_take(self.stage_n)
        self.out = [torch.empty((nray, max_rows, 8), dtype=F64, device=device) for _ in range(2)]
        # row 0 (the host initial rows) is every ray's "previous row" of chunk 1
        row0 = np.stack([np.ascontiguousarray(h[0]).reshape(-1) for h in hist], axis=1)
        self.last = torch.as_tensor(row0).to(device).view(torch.int64)       # [nray, 7] bits
        self.changed = [torch.empty(nray, dtype=torch.bool, device=device) for _ in range(2)]
        # each chunk's previous row travels with it (7 x nray doubles): the
        # host fill of a chunk then depends on no other chunk's
        self.prev_dev = [torch.empty((7, nray), dtype=F64, device=device) for _ in range(2)]
        self.prev_host = [torch.empty((7, nray), dtype=F64, pin_memory=True) for _ in range(2)]
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.futs = [[], []]
        self.pending = None
        self.gathered = [None, None]
        self.k = 0
        self.lock = threading.Lock()
        self.t_wait = self.t_fill = 0.0   # summed over tasks (diagnostic)
        self.shipped = 0          # rays x rows shipped over PCIe (diagnostic)
        self.delivered = 0

    def buffers(self):
        """The two device row buffers the engine alternates between."""
        return self.out

    def __call__(self, i0, i1, view):
        k, b = self.k, self.k % 2
        self.k += 1
        # the previous chunk first: its nonzero() waits for its compare only
        # (this launch is already queued, so the GPU stays busy meanwhile)
        if self.pending is not None:
            self._flush(*self.pending)
            self.pending = None
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(ready)
            bits = view[:, :, :7].view(torch.int64)
            self.prev_dev[b].copy_(self.last.t().view(F64))
            torch.any((bits != self.last[:, None, :]).reshape(self.nray, -1), dim=1, out=self.changed[b])
            self.last.copy_(bits[:, -1, :])
        self.pending = (b, i0, i1, view)
        # launch k+1 writes the buffer chunk k-1 was read from: its gather
        # was queued by the _flush above
        if self.gathered[1 - b] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.gathered[1 - b])
        if self.progress is not None:
            self.progress(i1 - 1)

    def _flush(self, b, i0, i1, view):
        r = i1 - i0
        # staging b and prev_host b were last read by chunk k-2's host tasks
        for f in self.futs[b]:
            f.result()
        with torch.cuda.stream(self.copy_stream):
            self.prev_host[b].copy_(self.prev_dev[b], non_blocking=True)
            cols = torch.nonzero(self.changed[b]).squeeze(1)     # syncs on this chunk's compare
            n = int(cols.numel())
            stage = self.stage_dev[b][: 7 * r * n].view(7, r, n)
            if n == self.nray:
                stage.copy_(view[:, :, :7].permute(2, 1, 0))
            elif n:
                stage.copy_(view.index_select(0, cols)[:, :, :7].permute(2, 1, 0))
            g = torch.cuda.Event()
            g.record(self.copy_stream)
            cols_h = cols.cpu().numpy() if 0 < n < self.nray else None
            host = self.stage_host[b][: 7 * r * n]
            d2h = []                 # one DMA per variable: its host fill starts when it lands
            for v in range(7):
                if n:
                    host[v * r * n:(v + 1) * r * n].copy_(stage[v].view(-1), non_blocking=True)
                d2h.append(torch.cuda.Event())
                d2h[-1].record(self.copy_stream)
        self.gathered[b] = g
        self.shipped += n * r
        self.delivered += self.nray * r
        src = host.numpy().reshape(7, r, n)
        prev = self.prev_host[b].numpy()
        step = max(1, -(-r * 7 // self.workers))
        self.futs[b] = [self.pool.submit(self._fill, d2h[v], src, prev[v], v, a, min(a + step, r), i0,
                                         cols_h)
                        for v in range(7) for a in range(0, r, step)]

    def _fill(self, ev, src, prev, v, a, e, i0, cols):
        t0 = time.perf_counter()
        ev.synchronize()
        t1 = time.perf_counter()
        self._fill_rows(src, prev, v, a, e, i0, cols)
        t2 = time.perf_counter()
        with self.lock:
            self.t_wait += t1 - t0
            self.t_fill += t2 - t1

    def _fill_rows(self, src, prev, v, a, e, i0, cols):
        h = self.hist[v]
        dst = h[i0 + a:i0 + e].reshape(e - a, self.nray)
        n = src.shape[2]
        if n == self.nray:
            dst[:] = src[v, a:e]
            return
        fill_rows(dst, prev, src[v, a:e], cols)

    def finish(self):
        if self.pending is not None:
            self._flush(*self.pending)
            self.pending = None
        for fs in self.futs:
            for f in fs:
                f.result()
        self.copy_stream.synchronize()
        self.pool.shutdown(wait=True)
        if self.stage_host is not None:
            _pinned_release(self.stage_n, self.stage_host)
            self.stage_host = None
