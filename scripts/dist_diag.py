"""Diagnose tests/test_gpu_dist.py: world-2 (gloo, one GPU) vs one process, per-key max-abs diffs,
for streams on/off and overlap on/off."""
import io
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

NETS = ("G1", "G2", "D1", "D2")


def batches():
    g = torch.Generator().manual_seed(21)
    return [tuple(torch.rand((4, c, 256, 256), generator=g) * 2 - 1 for c in (3, 1, 3)) for _ in range(2)]


def trainer(streams, overlap):
    from stcgan_amd.stcgan import STCGAN
    torch.manual_seed(5)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type="normal", ngf=16, dtype="bf16",
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None, streams=streams)
    tr = STCGAN(a)
    if not overlap:
        for s in (tr.sync_G, tr.sync_D):
            for h in s.hooks:
                h.remove()
            s.hooks, s.overlap = [], False
    return tr


def steps(tr, grads_out=None):
    for i, (x, m, y) in enumerate(batches()):
        if grads_out is not None and i == 0:
            st0 = tr.optim_D.step
            def cap():
                grads_out.update({f"D{j}.{n}": p.grad.detach().cpu().clone() for j, net in ((1, tr.D1), (2, tr.D2))
                                  for n, p in net.named_parameters()})
                st0()
            tr.optim_D.step = cap
        tr.train_step(x.cuda(), m.cuda(), y.cuda())
        if grads_out is not None and i == 0:
            tr.optim_D.step = st0
    torch.cuda.synchronize()
    return {n: {k: v.cpu() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}


SNAPS = []


def patch_launch():
    """Snapshot (async device clone) every flat bucket right after its gather, before the exchange."""
    from stcgan_amd import parallel
    orig_launch = parallel.GradAllReduce._launch
    orig_cat = torch.cat

    def launch(self, gi):
        def cat(ts, out=None):
            r = orig_cat(ts, out=out)
            SNAPS.append(out.clone())
            return r
        torch.cat = cat
        try:
            return orig_launch(self, gi)
        finally:
            torch.cat = orig_cat
    parallel.GradAllReduce._launch = launch


def worker(rank, port, streams, overlap, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    patch_launch()
    g = {}
    st = steps(trainer(streams, overlap), None)
    torch.cuda.synchronize()
    buf = io.BytesIO()
    torch.save({"st": st, "g": g, "snaps": [t.cpu() for t in SNAPS]}, buf)
    q.put((rank, buf.getvalue()))
    dist.barrier()
    dist.destroy_process_group()


def main():
    import socket
    for streams, overlap in ((True, False),) * 5:
        if True:
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            ps = [ctx.Process(target=worker, args=(r, port, streams, overlap, q)) for r in range(2)]
            for p in ps:
                p.start()
            got = dict(q.get(timeout=200) for _ in range(2))
            for p in ps:
                p.join(60)
            g1 = {}
            want = steps(trainer(streams, False), g1)
            d0 = torch.load(io.BytesIO(got[0]), weights_only=True)
            d1 = torch.load(io.BytesIO(got[1]), weights_only=True)
            diffs = [(i, float((a - b).abs().max())) for i, (a, b) in enumerate(zip(d0["snaps"], d1["snaps"]))]
            print(f"local gathered grads rank0 vs rank1: {len(d0['snaps'])} buckets, max diffs {diffs}", flush=True)
            tr0 = trainer(streams, False)
            order = [tr0.D2, tr0.D1, tr0.G2, tr0.G1]
            for bi, (a, b) in enumerate(zip(d0["snaps"], d1["snaps"])):
                net = order[bi % 4]
                off = 0
                for n, p in net.named_parameters():
                    k = p.numel()
                    da, db = a[off:off + k], b[off:off + k]
                    nd = int((da != db).sum())
                    if nd:
                        idx = (da != db).nonzero().flatten().tolist()
                        pos = [tuple(int(v) for v in torch.unravel_index(torch.tensor(i), tuple(p.shape))) for i in idx[:40]]
                        print(f"  positions {pos}", flush=True)
                        print(f"  bucket {bi} ({['D2', 'D1', 'G2', 'G1'][bi % 4]}) {n}: {nd}/{k} elements differ, "
                              f"max {float((da - db).abs().max()):.3e} |g| {float(da.abs().max()):.3e}", flush=True)
                    off += k
            del tr0
            print(f"== streams={streams} overlap={overlap}", flush=True)
            for r in (0, 1):
                d = torch.load(io.BytesIO(got[r]), weights_only=True)
                bad = []
                for k, v in g1.items():
                    if k not in d["g"]:
                        continue
                    e = float((d["g"][k] - v).abs().max())
                    if e > 0:
                        bad.append(f"grad {k} {e:.3e} (|g| {float(v.abs().max()):.3e})")
                for n in NETS:
                    for k, v in want[n].items():
                        if not torch.equal(d["st"][n][k], v):
                            bad.append(f"state {n}.{k} {float((d['st'][n][k].float() - v.float()).abs().max()):.3e}")
                print(f"rank {r}: {len(bad)} mismatches", *bad[:12], sep="\n  ", flush=True)


if __name__ == "__main__":
    main()
