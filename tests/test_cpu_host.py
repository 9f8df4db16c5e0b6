"""CPU-only tests: the C-ABI library loads and exports every symbol of include/vspike.h with the
struct layouts the binding mirrors; host logic (config loader, flat layout, DP exchange over gloo)
behaves like the reference.  No compute kernel is called here (no GPU in this container)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "video-spike_amd", "config")


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "vspike.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vs_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def built_lib():
    from vspike import build
    build.build(verbose=False)
    return build.LIB_PATH


def test_library_exports_every_header_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    syms = _header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    from vspike import _lib
    assert set(_lib.PROTOTYPES) == set(syms), set(syms) ^ set(_lib.PROTOTYPES)


def test_abi_struct_mirrors_and_version(built_lib):
    from vspike import _lib
    lib = _lib.lib()                       # verifies struct sizes against the C side
    assert lib.vs_version() >= 4
    assert lib.vs_struct_size(99) == -1


def test_build_id_matches_sources(built_lib):
    """vs_build_id() is the hash of the sources the loaded library was compiled from."""
    from vspike import _lib, build
    assert _lib.build_id() == build.source_hash()


def test_knobs_and_dispatch_counters_without_gpu(built_lib):
    """Knob overrides round-trip (read once from the environment, no getenv on launch paths);
    dispatch counters read and reset; unknown ids are rejected."""
    from vspike import _lib
    lib = _lib.lib()
    assert len(_lib.KNOB_NAMES) <= _lib.KNOB_COUNT and len(_lib.PATH_NAMES) <= _lib.PATH_COUNT
    prev = _lib.knob_set("wslab_g", 256)
    assert _lib.knob_get("wslab_g") == 256
    with _lib.knob("wslab_g", 128):
        assert _lib.knob_get("wslab_g") == 128
    assert _lib.knob_get("wslab_g") == 256
    _lib.knob_set("wslab_g", prev)
    assert lib.vs_knob_get(999) == -1 and lib.vs_knob_set(-1, 0) == -1
    _lib.dispatch_reset()
    assert set(_lib.dispatch_counts().values()) == {0}


def test_mse_criterion_selection():
    from vspike import make_criterion, mse_mean, poisson_nll_mean
    assert make_criterion(None) is poisson_nll_mean
    assert make_criterion({"training": {"loss": "mse"}}) is mse_mean
    assert make_criterion({"training": {}}) is poisson_nll_mean
    with pytest.raises(ValueError):
        make_criterion({"training": {"loss": "huber"}})


def test_gpu_only_entry_points_reject_bad_args_without_launching(built_lib):
    from vspike import _lib
    lib = _lib.lib()
    d = _lib.GemmDesc()
    d.dtype = 7
    assert lib.vs_gemm(ctypes.byref(d), None) == -1
    assert b"dtype" in lib.vs_last_error()
    assert lib.vs_attn_fwd(1, 1, 10, 1, 32, None, 192, None, 64, None, 0.125, None) == -1
    assert b"head dim" in lib.vs_last_error()
    # the gather weight gradient: null operands, then a tubelet it is not built for
    assert lib.vs_patch_embed_dw(2, 16, 3, 224, 224, 2, 16, None, None, 192, 192, None, 1536, None, None, 0, None) == -1
    assert b"null pointer" in lib.vs_last_error()
    buf = (ctypes.c_float * 64)()
    p = ctypes.addressof(buf)
    assert lib.vs_patch_embed_dw(2, 16, 3, 224, 224, 4, 16, p, p, 192, 192, p, 1536, None, p, 0, None) == -1
    assert b"tubelet 2" in lib.vs_last_error()
    assert lib.vs_patch_embed_dw(2, 16, 3, 224, 224, 2, 16, p, p, 96, 96, p, 1536, None, p, 0, None) == -1
    assert b"multiple of 64" in lib.vs_last_error()
    assert lib.vs_patch_embed_dw_workspace_bytes(200704, 192, 1536) > 0


def test_product_ops_refuse_cpu_tensors(built_lib):
    from vspike import ops
    from vspike._lib import VsError
    with pytest.raises(VsError):
        ops.cast(torch.zeros(8), torch.zeros(8, dtype=torch.bfloat16))


def test_config_loader_matches_reference(golden):
    from vspike.config import config_from_kwargs, load_run_config, update_config
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    for key, expected in ref.items():
        m, t = key.split("+")
        cfg = load_run_config(os.path.join(CFG, "model", m + ".yaml"), os.path.join(CFG, "train", t + ".yaml"))
        assert json.loads(json.dumps(cfg)) == expected, key
    c = config_from_kwargs({"a.b": "3", "a.c": "[1, 2]", "d": "null", "e": "1e-3", "f": "true"})
    assert c.a.b == 3 and c.a.c == [1, 2] and c.d is None and c.e == 1e-3 and c.f is True
    import argparse
    ns = argparse.Namespace(seed=7)
    assert update_config(ns, {"seed": 42}) == {"seed": 42}    # reference quirk: argparse values dropped


def test_vit_layout_covers_reference_names():
    from oracle import cpu_ref
    from vspike.layout import BackboneCfg, VitLayout, modern_name
    cfg = BackboneCfg(image_size=112, num_frames=8, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                      intermediate_size=512)
    lay = VitLayout(cfg, 64, 1600)
    names = [n for n, *_ in lay.hf_items()]
    # transformers 4.38 spelling (reference pin, env.yaml:30; modeling_videomae.py:216-218)
    assert "video_mae.encoder.layer.1.attention.attention.q_bias" in names
    assert "video_mae.encoder.layer.1.attention.attention.v_bias" in names
    ref = [n for n in cpu_ref.vit_param_shapes(cpu_ref.VIT_SMALL_FIXTURE, 64, 16)]   # newer HF spelling
    assert sorted(modern_name(n) for n in names) == sorted(ref)
    for s in list(lay.enc.slots.values()) + list(lay.head.slots.values()):
        assert s.offset % 64 == 0


def test_vit_module_builds_on_cpu_and_maps_weights():
    """Module construction and the reference-name weight mapping are host logic (no kernels)."""
    from oracle import cpu_ref
    from vspike import VideoMAE
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    conf = {"backbone": {"image_size": 112, "num_frames": 8, "hidden_size": 128, "num_hidden_layers": 2,
                         "num_attention_heads": 2, "intermediate_size": 512},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 1600}}
    m = VideoMAE(conf)
    assert not m.enc_flat.requires_grad        # reference default: frozen encoder (videomae.py:34-36)
    params = cpu_ref.make_vit_params(cfg, 64, 16)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    back = m.reference_state_dict(modern_names=True)
    for k, v in params.items():
        assert np.array_equal(back[k].numpy(), v), k
    with pytest.raises(Exception):
        m(torch.zeros(1, 8, 3, 112, 112))      # CPU tensor: no fallback path


def test_vit_loads_reference_era_checkpoint_names():
    """A state_dict saved by the reference (transformers 4.38: `q_bias` / `v_bias`, no key bias)
    loads strictly and round-trips; the newer names load to the same weights."""
    from oracle import cpu_ref
    from vspike import VideoMAE
    from vspike.layout import modern_name
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    conf = {"backbone": {"image_size": 112, "num_frames": 8, "hidden_size": 128, "num_hidden_layers": 2,
                         "num_attention_heads": 2, "intermediate_size": 512},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 1600}}
    params = cpu_ref.make_vit_params(cfg, 64, 16)
    legacy = {}
    m0 = VideoMAE(conf)
    for name, *_ in m0.layout.hf_items():
        legacy[name] = torch.from_numpy(params[modern_name(name)])
    assert any(k.endswith("attention.attention.q_bias") for k in legacy)
    m = VideoMAE(conf)
    m.load_reference_state_dict(legacy, strict=True)
    back = m.reference_state_dict()
    assert set(back) == set(legacy)
    for k, v in legacy.items():
        assert torch.equal(back[k], v), k
    m2 = VideoMAE(conf)
    m2.load_reference_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
    assert torch.equal(m.enc_flat, m2.enc_flat) and torch.equal(m.head_flat, m2.head_flat)
    with pytest.raises(KeyError):
        m.load_reference_state_dict({k: v for k, v in legacy.items() if not k.endswith("q_bias")}, strict=True)


def _dp_worker(rank, world, port, out):
    import torch.distributed as dist
    from vspike.dp import GradExchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Fake(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.enc_flat = torch.nn.Parameter(torch.zeros(1000))
            self.head_flat = torch.nn.Parameter(torch.zeros(300))
            self.extra = torch.nn.Parameter(torch.zeros(7))
            self.grad_sink = None

    m = Fake()
    with torch.no_grad():                          # replicas initialised differently ...
        m.enc_flat.fill_(10.0 + rank)
        m.extra.fill_(-rank)
    ex = GradExchange(m, bucket_mb=0.001)          # 262 elements per bucket -> several buckets
    init = (m.enc_flat.detach().clone(), m.extra.detach().clone())    # ... rank 0's after the broadcast
    gh = ex.grad_buffer(m.head_flat)
    gh += rank + 1
    ex.mark_ready(m.head_flat, 0, 300)
    ge = ex.grad_buffer(m.enc_flat)
    for lo in range(900, -1, -100):                # layers finish in reverse order
        ge[lo:lo + 100] += (rank + 1) * (lo + 1)
        ex.mark_ready(m.enc_flat, lo, lo + 100)
    m.extra.grad = torch.full((7,), float(rank))
    ex.finish()
    out[rank] = (m.head_flat.grad.clone(), m.enc_flat.grad.clone(), m.extra.grad.clone(), init)
    dist.destroy_process_group()


def test_grad_exchange_gloo_world2():
    import torch.multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_dp_worker, args=(2, port, out), nprocs=2, join=True)
    for r in range(2):
        h, e, x, (p_enc, p_extra) = out[r]
        assert torch.all(p_enc == 10.0) and torch.all(p_extra == 0.0)      # DDP-style broadcast from rank 0
        assert torch.all(h == 3.0)
        ref = torch.cat([torch.full((100,), 3.0 * (lo + 1)) for lo in range(0, 1000, 100)])
        assert torch.equal(e, ref)
        assert torch.all(x == 1.0)
