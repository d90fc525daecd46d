"""Request-level micro-batching behind the model object.

The unchanged AmenitiesDetector runs `self.model(**inputs)` once per image at batch 1
(reference serve.py:98-100, 180-181). Calls that arrive CONCURRENTLY — several Serve request
threads, or one request's images once the caller runs the model in a worker thread
(`await asyncio.to_thread(self.model, **inputs)`) — are coalesced here
into one engine forward: a single collector thread owns the device engine, takes up to
`max_batch` queued images of the same shape within `max_wait_ms` of the first, runs them as
one batch and hands each caller its own rows. Images never interact in the forward (every
kernel is per image / per query), so a caller gets what its own bs1 call computes up to fp32
summation order (bs1 GEMMs use split-K).
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future

import torch


class MicroBatcher:
    def __init__(self, run_batch, device, max_batch: int = 32, max_wait_ms: float = 2.0):
        """run_batch(pixel_values [B,3,H,W] on `device`) -> (logits [B,Q,C], boxes [B,Q,4])."""
        self._run = run_batch
        self.device = torch.device(device)
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1e3
        self._q: queue.Queue = queue.Queue()
        self._pending = 0  # submitted, not yet resolved: nobody beyond the taken ones → no wait
        self._pending_lock = threading.Lock()
        self.batches = 0  # engine forwards run (diagnostics / tests)
        self.images = 0
        self._thread = threading.Thread(target=self._loop, name="spotter-microbatcher", daemon=True)
        self._thread.start()

    def submit(self, pixel_values: torch.Tensor) -> Future:
        """Queue a [n,3,H,W] batch; the Future resolves to its (logits, boxes) rows (owned copies)."""
        fut: Future = Future()
        with self._pending_lock:
            self._pending += 1
        self._q.put((pixel_values, fut))
        return fut

    def __call__(self, pixel_values: torch.Tensor):
        return self.submit(pixel_values).result()

    def _others_waiting(self, taken: int) -> bool:
        """True while some submitted image is not among the `taken` ones: only then is waiting for
        more worth anything. (The collector resolves every future itself, so the count is exact.)"""
        with self._pending_lock:
            return self._pending > taken

    def _take(self):
        first = self._q.get()
        if first is None:
            return None
        items = [first]
        n = first[0].shape[0]
        shape = tuple(first[0].shape[1:])
        deadline = time.perf_counter() + self.max_wait
        held = []
        while n < self.max_batch:
            if not self._others_waiting(len(items)):
                break  # a lone serial caller (the unchanged serve.py) is dispatched at once
            left = deadline - time.perf_counter()
            if left <= 0:
                break
            try:
                it = self._q.get(timeout=left)
            except queue.Empty:
                break
            if it is None:
                held.append(it)
                break
            if tuple(it[0].shape[1:]) != shape or n + it[0].shape[0] > self.max_batch:
                held.append(it)  # another size, or no room: next batch
                break
            items.append(it)
            n += it[0].shape[0]
        for it in held:
            self._q.put(it)
        return items

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            items = self._take()
            if items is None:
                return
            outs, err = None, None
            try:
                xs = [x.to(self.device, non_blocking=True) for x, _ in items]
                x = xs[0] if len(xs) == 1 else torch.cat(xs, 0)
                logits, boxes = self._run(x)
                self.batches += 1
                self.images += x.shape[0]
                off = 0
                outs = []
                for (xi, fut) in items:
                    k = xi.shape[0]
                    outs.append((logits[off:off + k].clone(), boxes[off:off + k].clone()))
                    off += k
                if self.device.type == "cuda":
                    torch.cuda.current_stream().synchronize()
            except BaseException as e:  # every waiting caller sees the failure
                err = e
            finally:
                with self._pending_lock:
                    self._pending -= len(items)  # once per item, whatever happened
            for i, (_, fut) in enumerate(items):
                # each future on its own: a caller that cancelled its future (or one already resolved)
                # cannot fail the others or the collector thread
                try:
                    if err is not None:
                        fut.set_exception(err)
                    else:
                        fut.set_result(outs[i])
                except Exception:
                    pass

    def close(self):
        self._q.put(None)
        self._thread.join(timeout=10)
