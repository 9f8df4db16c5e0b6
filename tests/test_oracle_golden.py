"""Pin the CPU restatement (oracle/cpu_ref.py) to fixtures generated from the reference itself
(oracle/gen_fixtures.py).  Runs on CPU, no GPU, no /root/reference needed."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref, prng


def test_prng_is_deterministic_and_sane():
    a = prng.normal(3, (1000,), "x")
    b = prng.normal(3, (1000,), "x")
    c = prng.normal(3, (1000,), "y")
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    z = prng.normal(0, (200000,), "z")
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    y = prng.spike_targets(1, (4, 100, 16))
    assert y.min() >= 0 and np.all(y == np.round(y))


def test_linear_plugin_matches_reference(golden):
    fx = golden("linear_f.npz")
    B, T, HW, n = 4, 8, 64, 16
    shapes = cpu_ref.linear_param_shapes(T * HW * HW, [256, 128], 64, [128, 256], 100 * n)
    P = cpu_ref.to_torch(cpu_ref.make_linear_params(shapes))
    video = np.floor(prng.uniform(0, B * T * HW * HW, "video") * 256.0).astype(np.float32).reshape(B, T, 1, HW, HW)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    out = cpu_ref.linear_plugin_forward(torch.from_numpy(video), P)
    loss = cpu_ref.poisson_nll_mean(out, y)
    loss.backward()
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-5, atol=1e-5)
    assert abs(loss.item() - fx["loss"][0]) <= 1e-6 * abs(fx["loss"][0])
    for k, p in P.items():
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=1e-4, atol=1e-7)
        assert ok, msg


def test_linear_loss_curve_matches_reference(golden):
    fx = golden("linear_f.npz")
    B, T, HW, n = 4, 8, 64, 16
    shapes = cpu_ref.linear_param_shapes(T * HW * HW, [256, 128], 64, [128, 256], 100 * n)
    P = cpu_ref.to_torch(cpu_ref.make_linear_params(shapes))
    batches = []
    for s in range(5):
        v = np.floor(prng.uniform(100 + s, B * T * HW * HW, "video") * 256.0).astype(np.float32)
        batches.append((torch.from_numpy(v.reshape(B, T, 1, HW, HW)),
                        torch.from_numpy(prng.spike_targets(200 + s, (B, 100, n)))))
    curve = cpu_ref.train_curve(cpu_ref.linear_plugin_forward, P, batches, lr=1e-6)
    np.testing.assert_allclose(curve, fx["curve"], rtol=1e-5)


def _vit_small_setup(trainable_encoder=True):
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    return cfg, P, px, y


def test_vit_small_forward_backward_matches_reference(golden):
    fx = golden("vit_small.npz")
    cfg, P, px, y = _vit_small_setup()
    hid = cpu_ref.videomae_encoder(px, P, cfg)
    np.testing.assert_allclose(hid.detach().numpy(), fx["last_hidden"], rtol=1e-4, atol=1e-5)
    out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)
    loss = cpu_ref.poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    loss.backward()
    for k, p in P.items():
        if ".key.bias" in k:
            continue
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=2e-4, atol=1e-7)
        assert ok, msg


@pytest.mark.parametrize("frozen", [True, False])
def test_vit_small_loss_curve_matches_reference(golden, frozen):
    fx = golden("vit_small.npz")
    cfg, P, _, _ = _vit_small_setup()
    B, n = 2, 16
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=300 + s)),
                torch.from_numpy(prng.spike_targets(350 + s, (B, 100, n)))) for s in range(4)]
    fwd = lambda x, PP: cpu_ref.videomae_plugin_forward(x, PP, cfg, freeze_encoder=frozen)  # noqa: E731
    trainable = (lambda k: not k.startswith("video_mae.")) if frozen else None
    curve = cpu_ref.train_curve(fwd, P, batches, lr=1e-5, trainable=trainable)
    np.testing.assert_allclose(curve, fx["curve_frozen" if frozen else "curve_train"], rtol=1e-4)


def test_vit_tiny_full_tokens_matches_reference(golden):
    fx = golden("vit_tiny1l.npz")
    cfg = cpu_ref.ViTCfg(hidden_size=192, num_attention_heads=3, intermediate_size=768, num_hidden_layers=1)
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, 8), requires_grad=False)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 1))
    with torch.no_grad():
        hid = cpu_ref.videomae_encoder(px, P, cfg)
        out = cpu_ref.videomae_plugin_forward(px, P, cfg)
    ok, msg = cpu_ref.compare_summary("last_hidden", hid.numpy(), fx, rtol=1e-4, atol=1e-6)
    assert ok, msg
    np.testing.assert_allclose(out.numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)


def test_vit_tiny12_bench_geometry_matches_reference(golden):
    """The bench geometry (C2: ViT-Tiny, 12 layers, 1568 tokens, n=128, trainable encoder), B=2:
    log-rates, last hidden state and every gradient, plus the 4-step train curve."""
    fx = golden("vit_tiny12.npz")
    cfg, B, n = cpu_ref.VIT_TINY, 2, 128
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    hid = cpu_ref.videomae_encoder(px, P, cfg)
    ok, msg = cpu_ref.compare_summary("last_hidden", hid.detach().numpy(), fx, rtol=1e-4, atol=1e-6)
    assert ok, msg
    out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)
    loss = cpu_ref.poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    loss.backward()
    for k, p in P.items():
        if ".key.bias" in k:
            continue
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=5e-4, atol=1e-7)
        assert ok, msg
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=400 + s)),
                torch.from_numpy(prng.spike_targets(450 + s, (B, 100, n)))) for s in range(4)]
    fwd = lambda x, PP: cpu_ref.videomae_plugin_forward(x, PP, cfg, freeze_encoder=False)  # noqa: E731
    curve = cpu_ref.train_curve(fwd, P, batches, lr=1e-6)
    np.testing.assert_allclose(curve, fx["curve_train"], rtol=1e-4)


def test_vit_tiny12_bench_batch_matches_reference(golden):
    """The bench's exact batch (C2, 12 layers, B=16 -> 25,088 token rows, fixture vit_tiny12_b16):
    log-rates, loss, every gradient and the 3-step train curve."""
    fx = golden("vit_tiny12_b16.npz")
    cfg, B, n = cpu_ref.VIT_TINY, 16, 128
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=16))
    y = torch.from_numpy(prng.spike_targets(16, (B, 100, n)))
    out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)
    loss = cpu_ref.poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    loss.backward()
    for k, p in P.items():
        if ".key.bias" in k:
            continue
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=5e-4, atol=1e-7)
        assert ok, msg
    del out, loss
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=600 + s)),
                torch.from_numpy(prng.spike_targets(650 + s, (B, 100, n)))) for s in range(3)]
    fwd = lambda x, PP: cpu_ref.videomae_plugin_forward(x, PP, cfg, freeze_encoder=False)  # noqa: E731
    curve = cpu_ref.train_curve(fwd, P, batches, lr=1e-6)
    np.testing.assert_allclose(curve, fx["curve_train"], rtol=1e-4)


def test_vit_base_32_frames_matches_reference(golden):
    """BASELINE C5's encoder geometry (videomae-base, 32 frames -> 3,136 tokens, n=1024), 1 layer, B=1."""
    fx = golden("vit_base32f.npz")
    cfg, B, n = cpu_ref.ViTCfg(num_frames=32, num_hidden_layers=1), 1, 1024
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=32))
    y = torch.from_numpy(prng.spike_targets(32, (B, 100, n)))
    out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)
    loss = cpu_ref.poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    loss.backward()
    for k, p in P.items():
        if ".key.bias" in k:
            continue
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=5e-4, atol=1e-7)
        assert ok, msg


def test_vit_base_one_layer_matches_reference(golden):
    """The reference plugin's real width (videomae-base d768 / 12 heads, C3's n=512), 1 layer, B=1:
    trainable fwd+bwd, and the default frozen-encoder curve."""
    fx = golden("vit_base1l.npz")
    cfg, B, n = cpu_ref.ViTCfg(num_hidden_layers=1), 1, 512
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    np.testing.assert_allclose(out.detach().numpy(), fx["log_rates"], rtol=1e-4, atol=1e-5)
    loss = cpu_ref.poisson_nll_mean(out, y)
    loss.backward()
    assert abs(loss.item() - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    for k, p in P.items():
        if ".key.bias" in k:
            continue
        ok, msg = cpu_ref.compare_summary(k, p.grad.numpy(), fx, rtol=5e-4, atol=1e-7)
        assert ok, msg
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=500 + s)),
                torch.from_numpy(prng.spike_targets(550 + s, (B, 100, n)))) for s in range(3)]
    fwd = lambda x, PP: cpu_ref.videomae_plugin_forward(x, PP, cfg, freeze_encoder=True)  # noqa: E731
    curve = cpu_ref.train_curve(fwd, P, batches, lr=2e-7, trainable=lambda k: not k.startswith("video_mae."))
    np.testing.assert_allclose(curve, fx["curve_frozen"], rtol=1e-4)


def test_vit_base_two_layers_b16_forward_matches_reference(golden):
    """C3's benched-dispatch fixture (videomae-base, 2 layers, B=16, n=512; vit_base2l_b16): log-rates
    are per clip, so the oracle's forward of the first two clips pins it against the reference's
    (the full-batch backward is the GPU test's job: ~90 s of CPU here)."""
    fx = golden("vit_base2l_b16.npz")
    cfg, n = cpu_ref.ViTCfg(num_hidden_layers=2), 512
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n), requires_grad=False)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 16, seed=768))[:2]
    with torch.no_grad():
        out = cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False)
    ref = fx["log_rates"][:2]
    # the head input is 1,204,224 wide: summation-order noise ~1e-5 absolute on values near zero
    assert np.abs(out.numpy() - ref).max() <= 1e-5 * np.abs(ref).max() + 2e-5


def test_k0_preprocess_oracle_matches_reference_processor(golden):
    """K0 (videomae.py:18-25): the restated PIL bilinear resize + HF rescale/normalise reproduce the
    HF image processor's output bit for bit (fixture made by oracle/gen_fixtures.py gen_k0)."""
    import numpy as np
    from oracle import cpu_ref, prng
    fx = golden("k0_preprocess.npz")
    video = prng.video_frames(int(fx["seed"]), tuple(int(v) for v in fx["shape"]))
    idx = cpu_ref.frame_indices()
    assert np.array_equal(idx, fx["idx"])
    pv = cpu_ref.video_preprocess(video, idx, 224, fx["mean"], fx["std"])
    m0, s0 = np.float32(fx["mean"][0]), np.float32(fx["std"][0])
    for j, f in enumerate(fx["u8_frames"]):      # exact uint8 resize planes of the reference path
        u8 = fx["u8"][j].astype(np.float64)
        assert np.array_equal(((u8 * (1 / 255)).astype(np.float32) - m0) / s0, pv[0, f, 0])
    cpu_ref.compare_summary("pixel_values", pv, fx, rtol=1e-7, atol=0.0)


def test_metrics_restatement_matches_reference(golden):
    """oracle.metrics_ref (numpy, f32 like the reference) against outputs of the reference's own
    metrics_list / bits_per_spike (utils.py:122-167, metric_utils.py:36-102) on the same inputs."""
    import warnings
    from oracle import metrics_ref as M
    fx = golden("metrics.npz")
    warnings.simplefilter("ignore", RuntimeWarning)
    for name, (R, T, N, seed, mets, log_input) in M.METRIC_CASES.items():
        gt, pred = M.metric_case(name)
        if log_input:
            res = M.eval_session(gt, pred, mets)
        else:
            res = M.metrics_list(np.swapaxes(gt, -1, 0), np.swapaxes(pred, -1, 0), mets)
        for k in mets:
            assert abs(res[k] - float(fx[f"{name}.{k}"])) <= 1e-7, (name, k, res[k], fx[f"{name}.{k}"])
        if "bps" in mets:
            rates = np.exp(pred) if log_input else pred
            want = fx[f"{name}.bps_per_neuron"].copy()
            want[np.isinf(want)] = np.nan                   # utils.py:130-131
            got = M.per_neuron_bps(gt, rates.astype(np.float32))
            assert np.array_equal(np.isnan(got), np.isnan(want))
            np.testing.assert_allclose(got[~np.isnan(got)], want[~np.isnan(want)], rtol=1e-5, atol=2e-6)
    assert str(fx["m_wide.bps_error"]).startswith("IndexError")
