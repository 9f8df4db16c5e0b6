"""K0 on the device (videomae.py:10-11, 18-25): vs_video_preprocess against the CPU restatement
(oracle/cpu_ref.video_preprocess, itself pinned to the HF image processor by
tests/golden/k0_preprocess.npz).  Integer/byte work: the bar is bit-exact."""
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


def test_k0_matches_reference_fixture_bit_exact(golden):
    from vspike import ops
    fx = golden("k0_preprocess.npz")
    video = prng.video_frames(int(fx["seed"]), tuple(int(v) for v in fx["shape"]))
    out = ops.video_preprocess(torch.from_numpy(video).to(DEV), fx["idx"].tolist(), 224, fx["mean"], fx["std"])
    pv = out.cpu().numpy()
    m0, s0 = np.float32(fx["mean"][0]), np.float32(fx["std"][0])
    for j, f in enumerate(fx["u8_frames"]):
        want = ((fx["u8"][j].astype(np.float64) * (1 / 255)).astype(np.float32) - m0) / s0
        assert np.array_equal(pv[0, f, 0], want)
    cpu_ref.compare_summary("pixel_values", pv, fx, rtol=1e-7, atol=0.0)
    ref = cpu_ref.video_preprocess(video, fx["idx"], 224, fx["mean"], fx["std"])
    assert np.array_equal(pv, ref)


@pytest.mark.parametrize("h,size,t,nf", [(128, 224, 120, 16), (100, 224, 40, 5), (300, 224, 9, 3), (64, 64, 7, 7),
                                         (224, 112, 3, 2)])
def test_k0_shapes_bit_exact_vs_oracle(h, size, t, nf):
    """up-sampling (non-integer ratios), down-sampling (wider filter support), identity size."""
    from vspike import ops
    video = prng.video_frames(5 + h, (2, t, 1, h, h))
    idx = cpu_ref.frame_indices(nf, t)
    mean, std = (0.5, 0.45, 0.4), (0.25, 0.2, 0.3)
    out = ops.video_preprocess(torch.from_numpy(video).to(DEV), idx.tolist(), size, mean, std).cpu().numpy()
    ref = cpu_ref.video_preprocess(video, idx, size, mean, std)
    assert np.array_equal(out, ref), np.abs(out - ref).max()


def test_k0_uint8_input_equals_float_input():
    from vspike import ops
    video = prng.video_frames(3, (3, 30, 1, 128, 128))
    idx = cpu_ref.frame_indices(16, 30).tolist()
    a = ops.video_preprocess(torch.from_numpy(video).to(DEV), idx)
    b = ops.video_preprocess(torch.from_numpy(video.astype(np.uint8)).to(DEV), idx)
    assert torch.equal(a, b)


def test_k0_rejects_bad_arguments():
    from vspike import ops, _lib as L
    v = torch.zeros(1, 10, 1, 32, 32, device=DEV)
    with pytest.raises(L.VsError):
        ops.video_preprocess(v, [0, 10])                      # frame index out of range
    with pytest.raises(L.VsError):
        ops.video_preprocess(torch.zeros(1, 10, 1, 32, 16, device=DEV), [0])   # non-square frames


def test_videomae_forward_accepts_raw_video():
    """The plugin's forward takes the loader's raw (B, 120, 1, 128, 128) video, as the reference's does."""
    from vspike import VideoMAE
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    conf = {"model_class": "VideoMAE", "freeze_encoder": False, "compute_dtype": "fp32",
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size",
                                                       "layer_norm_eps")},
            "encoder": {"output_dim": 16}, "decoder": {"output_dim": 100 * 4}}
    m = VideoMAE(conf).to(DEV)
    video = prng.video_frames(9, (2, 120, 1, 128, 128))
    idx = cpu_ref.frame_indices(cfg.num_frames, 120)
    pv = cpu_ref.video_preprocess(video, idx, cfg.image_size, m.pp_mean, m.pp_std)
    with torch.no_grad():
        a = m(torch.from_numpy(video).to(DEV))
        b = m(torch.from_numpy(pv).to(DEV))
    assert torch.equal(a, b)


def test_shard_loader_to_device_feeds_the_plugin(tmp_path):
    """Shard -> pinned host -> async H2D (uint8) -> the VideoMAE plugin's raw-video path: the batch
    arrives intact and the uint8 frames give exactly the output of the same frames as float32
    (the reference's loader hands the model `.float()` frames, src/loader/base.py:41)."""
    from vspike.data import ShardLoader, write_shard
    from vspike import VideoMAE
    n, T, H = 4, 20, 64
    video = (prng.uniform(77, n * T * H * H, "v") * 256).astype(np.uint8).reshape(n, T, 1, H, H)
    ap = prng.spike_targets(78, (n, 100, 16))
    p = str(tmp_path / "s.vss")
    write_shard(p, video, ap, [f"e{i % 2}_{i}" for i in range(n)])
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    conf = {"model_class": "VideoMAE", "freeze_encoder": True, "compute_dtype": "fp32",
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size",
                                                       "layer_norm_eps")},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 1600}}
    m = VideoMAE(conf).to(DEV)
    got = 0
    for b in ShardLoader([p], batch_size=2, shuffle=False, device=DEV):
        idx = [int(k.split("_")[1]) for k in b["__key__"]]
        assert b["video"].is_cuda and b["video"].dtype == torch.uint8
        assert np.array_equal(b["video"].cpu().numpy(), video[idx])
        assert np.array_equal(b["ap"].cpu().numpy(), ap[idx])
        with torch.no_grad():
            assert torch.equal(m(b["video"]), m(b["video"].float()))
        got += len(idx)
    assert got == n
