"""Which part of the train step does a HIP-graph capture choke on?  Each variant captures one train step
(STCGAN.capture) in a fresh subprocess and replays it twice: single stream, + weight-gradient side
streams, + discriminator lanes, with and without the optimiser inside the graph.

  python scripts/graph_capture_probe.py            # all variants (subprocesses)
  python scripts/graph_capture_probe.py VARIANT    # one variant in this process
"""
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = ["one_stream", "wgrad_lane", "lanes", "lanes_no_optim", "lanes_ngf16_fp32", "lanes_forward_only",
            "lanes_no_wgrad_lane", "lanes_side"]


def run(variant):
    sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
    import torch
    from stcgan_amd import engine
    from stcgan_amd.stcgan import STCGAN
    engine.WGRAD_OVERLAP = variant not in ("one_stream", "lanes_no_wgrad_lane")
    engine.SIDE_IN_CAPTURE = variant == "lanes_side"  # the lanes' weight-gradient side streams kept in the capture
    ngf, dt = (16, "fp32") if variant.endswith("fp32") else (64, "bf16")
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type="normal", ngf=ngf, dtype=dt,
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None, streams=variant.startswith("lanes"))
    tr = STCGAN(a)
    if variant == "lanes_no_optim":
        tr.optim_D.step = tr.optim_G.step = lambda: None
    B = 4
    x = torch.rand((B, 3, 256, 256), device="cuda") * 2 - 1
    m = (torch.rand((B, 1, 256, 256), device="cuda") < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), device="cuda") * 2 - 1
    if variant == "lanes_forward_only":  # D lanes, no backward: the validation step
        tr.train_step(x, m, y)
        for n in ("G1", "G2", "D1", "D2"):
            getattr(tr, n).train()
        main = torch.cuda.current_stream()
        cap = torch.cuda.Stream()
        cap.wait_stream(main)
        with torch.cuda.stream(cap):
            tr.train_step(x, m, y, training=False)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        tr._lanes_stale = True
        with torch.cuda.graph(g, stream=cap):
            tr.train_step(x, m, y, training=False)
        g.replay()
        torch.cuda.synchronize()
        print(f"{variant}: captured and replayed", flush=True)
        return
    replay = tr.capture(x, m, y)
    replay()
    replay()
    torch.cuda.synchronize()
    print(f"{variant}: captured and replayed", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for v in VARIANTS:
            env = dict(os.environ)
            if os.environ.get("PROBE_LOG") and v.startswith("lanes"):
                env["AMD_LOG_LEVEL"] = os.environ["PROBE_LOG"]
            r = subprocess.run([sys.executable, "-u", __file__, v], capture_output=True, text=True, timeout=240, env=env)
            lines = (r.stdout + r.stderr).strip().splitlines()
            tail = [ln for ln in lines if "rror" in ln or "apture" in ln][-12:] + lines[-4:]
            print(f"== {v}: rc={r.returncode}", *tail, sep="\n  ", flush=True)
