"""Data parallel and the reference's real caller, on the GPU through the HIP path.

* GradExchange (vspike.dp) driven by the REAL VideoMAE backward (deferred side-stream joins,
  mark_ready ranges in reverse layer order): two ranks on one GPU over gloo, each on its half of a
  batch; the exchanged gradient / world must equal the single-process gradient of the whole batch
  (the reference's DP is accelerate -> DDP, src/train.py:61-64).
* torch DDP — what `accelerator.prepare` wraps a model in when launched multi-process — around the
  plugin, as is (DDP's own all-reduce at the end of the backward) and with `vspike.dp.attach_ddp`
  (the all-reduce overlapped with the backward through a DDP communication hook).
* accelerate itself at world size 1: `Accelerator().prepare(model, optimizer, scheduler)` and
  `accelerator.backward(loss)` (src/train.py:61-64, src/trainer/base.py:150) reproduce the
  reference's loss curve; the unwrapped module survives torch.save / torch.load (base.py:212,285-291).
Two ranks share cuda:0 (RCCL refuses two ranks on one device, so these use gloo; the RCCL path is
the same code with backend "nccl", exercised by bench.py --gpus N).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cfg(layers):
    return cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=128, num_hidden_layers=layers,
                          num_attention_heads=2, intermediate_size=512)


def _model(cfg, dtype, n=16, freeze=False):
    from vspike import VideoMAE
    conf = {"model_class": "VideoMAE", "freeze_encoder": freeze, "compute_dtype": dtype,
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size")},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    m = VideoMAE(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_vit_params(cfg, 64, n).items()})
    return m


def _batch(cfg, B=4, n=16, step=0):
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=700 + step))
    y = torch.from_numpy(prng.spike_targets(750 + step, (B, 100, n)))
    return px, y


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, layers, dtype, out):
    import torch.distributed as dist
    from vspike import poisson_nll_mean
    from vspike.dp import GradExchange, attach_ddp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(layers)
    torch.manual_seed(100 + rank)                  # replicas built differently: the broadcast aligns them
    m = _model(cfg, dtype)
    if rank == 1:
        with torch.no_grad():
            m.head_flat.add_(0.5)
    per = 4 // world
    if mode == "exchange":
        ex = GradExchange(m, bucket_mb=0.25)        # ~65 K floats per bucket: many buckets in flight
        net = m
    else:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(m, device_ids=[0])
        ex = attach_ddp(net, bucket_mb=0.25) if mode.startswith("ddp_attach") else None
    for step in range(2):                           # DDP rebuilds its buckets after the first step
        px, y = _batch(cfg, step=step)
        m.zero_grad(set_to_none=True)
        xs, ys = px[rank * per:(rank + 1) * per].to(DEV), y[rank * per:(rank + 1) * per].to(DEV)
        if mode.startswith("ddp_attach_accum"):
            # gradient accumulation: one clip per micro-batch, the first under no_sync (local only)
            for j in range(per):
                if j < per - 1 and mode == "ddp_attach_accum_split":
                    # forward under no_sync, backward outside it: DDP decides at forward time
                    with net.no_sync():
                        lj = poisson_nll_mean(net(xs[j:j + 1]), ys[j:j + 1])
                    lj.backward()
                elif j < per - 1:
                    with net.no_sync():
                        poisson_nll_mean(net(xs[j:j + 1]), ys[j:j + 1]).backward()
                else:
                    poisson_nll_mean(net(xs[j:j + 1]), ys[j:j + 1]).backward()
            continue
        loss = poisson_nll_mean(net(xs), ys)
        loss.backward()
        if mode == "exchange":
            ex.finish()
    torch.cuda.synchronize()
    # DDP averages over ranks; the exchange sums; accumulation sums `per` one-clip mean losses
    scale = 1.0 / world if mode == "exchange" else (1.0 / per if mode.startswith("ddp_attach_accum") else 1.0)
    out[rank] = (m.enc_flat.grad.detach().cpu() * scale, m.head_flat.grad.detach().cpu() * scale)
    dist.destroy_process_group()


def _single_process_grads(layers, dtype):
    from vspike import poisson_nll_mean
    cfg = _cfg(layers)
    m = _model(cfg, dtype)
    px, y = _batch(cfg, step=1)
    m.zero_grad(set_to_none=True)
    poisson_nll_mean(m(px.to(DEV)), y.to(DEV)).backward()
    torch.cuda.synchronize()
    return m.enc_flat.grad.detach().cpu(), m.head_flat.grad.detach().cpu(), m.layout


def _worst_slots(layout, got, want, k=4):
    """The parameter slots whose gradients differ most (for the failure message)."""
    errs = []
    for name, s in layout.slots.items():
        g, w = got[s.offset:s.offset + s.numel], want[s.offset:s.offset + s.numel]
        errs.append((float((g - w).norm() / w.norm().clamp_min(1e-30)), name))
    return sorted(errs, reverse=True)[:k]


@pytest.mark.parametrize("mode,layers,dtype,tol", [
    ("exchange", 2, "fp32", 1e-5),
    ("exchange", 4, "bf16", 1e-4),        # 4 layers: consecutive deferred joins (VS_BWD_DEFER_LAST)
    ("ddp", 2, "fp32", 1e-5),
    ("ddp", 4, "bf16", 1e-4),
    ("ddp_attach", 2, "fp32", 1e-5),
    ("ddp_attach", 4, "bf16", 1e-4),
    ("ddp_attach_accum", 2, "fp32", 1e-5),   # DDP no_sync micro-steps + attach_ddp
    ("ddp_attach_accum_split", 2, "fp32", 1e-5),   # forward in no_sync, backward outside
])
def test_two_ranks_equal_single_process_batch(mode, layers, dtype, tol):
    import torch.multiprocessing as mp
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), mode, layers, dtype, out), nprocs=world, join=True)
    ge, gh, lay = _single_process_grads(layers, dtype)
    for r in range(world):
        e, h = out[r]
        for got, want, what, ly in ((e, ge, "encoder", lay.enc), (h, gh, "head", lay.head)):
            err = float((got - want).norm() / want.norm())
            print(f"\n[{mode} {dtype} rank {r}] {what} grad rel err {err:.2e}")
            if err >= tol:   # which slots, and is the single-process reference itself reproducible?
                ge2 = _single_process_grads(layers, dtype)[0]
                assert err < tol, (mode, r, what, err, _worst_slots(ly, got, want),
                                   "ranks equal", torch.equal(out[0][0], out[1][0]),
                                   "single-process rerun equal", torch.equal(ge2, ge))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_accelerate_prepare_backward_and_checkpoint(golden, tmp_path):
    """The reference's caller, unchanged: Accelerator().prepare(model, optimizer, lr_scheduler)
    (src/train.py:61-64) and accelerator.backward(loss) (src/trainer/base.py:150) over 4 steps of
    the vit_small fixture's trainable-encoder curve; then the whole-module checkpoint of
    base.py:285-291 (torch.save({'model': module, 'epoch'})) reloads and computes the same outputs."""
    from accelerate import Accelerator
    from vspike import FusedAdamW, poisson_nll_mean
    fx = golden("vit_small.npz")
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _model(cfg, "fp32", n)
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=4, max_lr=1e-5, pct_start=0.15, div_factor=10)
    accelerator = Accelerator()
    model, optimizer, lr_scheduler = accelerator.prepare(m, opt, sched)
    losses = []
    for s in range(4):
        px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=300 + s)).to(accelerator.device)
        y = torch.from_numpy(prng.spike_targets(350 + s, (B, 100, n))).to(accelerator.device)
        loss = poisson_nll_mean(model(px), y)
        accelerator.backward(loss)
        optimizer.step()
        lr_scheduler.step()
        optimizer.zero_grad()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, fx["curve_train"], rtol=1e-3)
    module = accelerator.unwrap_model(model)
    torch.save({"model": module, "epoch": 3}, tmp_path / "model_best.pt")
    back = torch.load(tmp_path / "model_best.pt", weights_only=False)["model"]   # our own file
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=9)).to(DEV)
    with torch.no_grad():
        a, b = module(px), back(px)
    assert (a - b).abs().max().item() <= 1e-6 * a.abs().max().item()


def test_bench_gpus_2_launches_two_ranks_in_sync():
    """`bench.py --gpus 2` started WITHOUT a launcher spawns two ranks itself (the driver's scaling
    run calls it either way); gloo lets both share this box's one GPU.  Rank 0 prints the one JSON
    line with n_gpus = 2, the whole-job batch, and the replicas' weights equal after the steps."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--profile-steps", "0", "--batch", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = lines[0]
    print("\n", {k: line[k] for k in ("n_gpus", "value", "ms_per_step", "replicas_equal", "backend")})
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 4 and line["config"]["parallelism"] == "dp2"
    assert line["replicas_equal"] is True and line["value"] > 0


def test_rccl_comm_c_abi_single_rank():
    """vs_comm_* (the C-ABI exchange for non-Python hosts): one rank on this box's GPU — id, init,
    the in-place bucket all-reduce on the current stream (a sum over one rank is the identity,
    f32 and bf16, a 0-length bucket is a no-op), finalize."""
    from vspike.comm import RcclComm
    comm = RcclComm(1, 0, RcclComm.unique_id())
    for dt in (torch.float32, torch.bfloat16):
        t = torch.randn(1 << 20, device=DEV).to(dt)
        ref = t.clone()
        comm.allreduce_(t)
        torch.cuda.synchronize()
        assert torch.equal(t, ref)
    comm.allreduce_(torch.empty(0, device=DEV))
    comm.close()


# ------------------------------------------------------------------------------------------------
# R3D (BASELINE C4) under the exchange: the plugin hands each conv unit's span of its gradient buffer
# over as soon as that unit's backward has run (reverse order), so buckets all-reduce under the
# earlier units' backward (src/train.py:61-64, src/trainer/base.py:150)
# ------------------------------------------------------------------------------------------------
def _r3d(n=16):
    from vspike import R3D
    cfg = cpu_ref.R3DCfg(num_frames=4, image_size=56)
    conf = {"model_class": "R3D", "compute_dtype": "fp32", "freeze_encoder": False,
            "backbone": {"num_frames": cfg.num_frames, "image_size": cfg.image_size, "num_channels": cfg.num_channels},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    m = R3D(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_r3d_params(cfg, 64, n).items()},
                                strict=False)
    return cfg, m


def _r3d_batch(cfg, n=16):
    px = torch.from_numpy(cpu_ref.make_r3d_pixels(cfg, 4, seed=31))
    y = torch.from_numpy(prng.spike_targets(32, (4, 100, n)))
    return px, y


def _worker_r3d(rank, world, port, out):
    import torch.distributed as dist
    from vspike import poisson_nll_mean
    from vspike.dp import GradExchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, m = _r3d()
    if rank == 1:                                   # different replicas: the broadcast aligns them
        with torch.no_grad():
            m.enc_flat.mul_(1.5)
    ex = GradExchange(m, bucket_mb=0.25)
    px, y = _r3d_batch(cfg)
    per = 4 // world
    loss = poisson_nll_mean(m(px[rank * per:(rank + 1) * per].to(DEV)), y[rank * per:(rank + 1) * per].to(DEV))
    loss.backward()
    launched_in_backward = len(ex._works)           # collectives started before the backward returned
    ex.finish()
    torch.cuda.synchronize()
    out[rank] = (m.enc_flat.grad.detach().cpu() / world, m.head_flat.grad.detach().cpu() / world,
                 launched_in_backward)
    dist.destroy_process_group()


def test_r3d_two_ranks_exchange_overlaps_and_matches():
    """Two ranks (gloo, one GPU) each train the R3D plugin on half of a 4-clip batch with the exchange.
    Training-mode BatchNorm normalises by each rank's own batch (DDP without SyncBatchNorm does the
    same), so the reference is the average of the two halves' single-process gradients.  The
    per-unit hand-off must have launched several all-reduces before the backward returned."""
    import torch.multiprocessing as mp
    from vspike import poisson_nll_mean
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_r3d, args=(world, _free_port(), out), nprocs=world, join=True)
    cfg, m = _r3d()
    px, y = _r3d_batch(cfg)
    ge, gh = 0.0, 0.0
    for h in range(2):
        m.zero_grad(set_to_none=True)
        poisson_nll_mean(m(px[2 * h:2 * h + 2].to(DEV)), y[2 * h:2 * h + 2].to(DEV)).backward()
        torch.cuda.synchronize()
        ge = ge + m.enc_flat.grad.detach().cpu() / 2
        gh = gh + m.head_flat.grad.detach().cpu() / 2
    for r in range(world):
        e, h, launched = out[r]
        ee = float((e - ge).norm() / ge.norm())
        eh = float((h - gh).norm() / gh.norm())
        print(f"\n[r3d exchange rank {r}] encoder {ee:.2e} head {eh:.2e}, {launched} all-reduces launched "
              "during the backward")
        assert ee < 1e-5 and eh < 1e-5
        assert launched >= 4
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
