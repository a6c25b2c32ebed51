"""The north-star kernel set -- one train-mode G1+G2 forward at bs=32 256x256 -- timed three ways:
eager (HIP events over back-to-back forwards), host enqueue time of one forward while the GPU is
busy (is the eager number host-bound?), and one forward captured as a HIP graph and replayed.
Under ``rocprofv3 --kernel-trace`` the last ``--reps`` eager forwards give the per-kernel timeline
(scripts/fwd_timeline_read.py).  usage: fwd_timeline.py [--dtype bf16] [--reps 3] [--no-graph]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import networks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g1 = networks.get_generator(3, 1).apply(networks.weights_init).to(dev).set_compute_dtype(a.dtype).train()
    g2 = networks.get_generator(4, 3).apply(networks.weights_init).to(dev).set_compute_dtype(a.dtype).train()
    x = torch.rand((a.batch, 3, 256, 256), device=dev) * 2 - 1
    res = {}

    def fwd():
        m = g1(x)
        return g2([x, m])

    with torch.no_grad():
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        # host enqueue of one forward with the GPU busy (a spin kernel queued ahead)
        torch.cuda._sleep(200_000_000)
        t0 = time.perf_counter()
        fwd()
        res["host_enqueue_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fwd()
        e1.record()
        e1.synchronize()
        res["eager_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
        if not a.no_graph:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fwd()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    fwd()
            torch.cuda.synchronize()
            for _ in range(2):
                g.replay()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            e1.synchronize()
            res["graph_ms"] = round(e0.elapsed_time(e1) / a.reps, 4)
    flops = 770.95e9 * a.batch / 32
    for k in ("eager_ms", "graph_ms"):
        if k in res:
            res[k.replace("_ms", "_frac")] = round(flops / (res[k] * 1e-3) / 2516e12, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
