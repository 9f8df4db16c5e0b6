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
