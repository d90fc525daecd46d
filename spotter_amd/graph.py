"""hipGraph capture of one forward per (batch, height, width) — the /detect latency path.

At batch 1 the forward is ~250 short kernels, so host launch overhead dominates
(MI355X_MICROARCH.md, graph-replay-floor / boundary rows). The whole forward is
captured once with torch.cuda.CUDAGraph on the stream the C-ABI launches on and
replayed; the input is copied into the graph's static buffer first.
"""
from __future__ import annotations

import torch


class GraphRunner:
    def __init__(self, engine, batch: int, height: int, width: int, warmup: int = 2):
        self.engine = engine
        dev = engine.dev
        self.x = torch.zeros((batch, 3, height, width), dtype=torch.float32, device=dev)
        # The graph bakes in buffer addresses, so it gets a private workspace that no eager call
        # can reallocate (engine._ws / engine._outs are swapped in only while capturing).
        self.ws, self.outs = {}, {}
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        saved = engine._ws, engine._outs
        engine._ws, engine._outs = self.ws, self.outs
        try:
            with torch.cuda.stream(side):
                for _ in range(warmup):  # allocate workspaces / constants outside capture
                    engine.forward(self.x, microbatches=1)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            # thread_local: request threads may keep launching (processor uploads) while the batcher
            # thread captures; their work is on other streams and is not part of this graph
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.logits, self.boxes = engine.forward(self.x, microbatches=1)
        finally:
            engine._ws, engine._outs = saved

    def __call__(self, pixel_values: torch.Tensor):
        self.x.copy_(pixel_values, non_blocking=True)
        self.graph.replay()
        return self.logits, self.boxes
