"""Parity bars shared by the GPU tests and bench.py's parity legs (TEST INFRASTRUCTURE ONLY: the
product path never imports this package).

MX-FP8 (BASELINE C5, compute_dtype "fp8"): e4m3 keeps 3 mantissa bits (2^-4 relative per element,
16x bf16's), so the block outputs carry ~1-2 % relative noise.  Bars ~2x the values measured on
MI355X against the vit_base32f fixture (1 layer, 3,136 tokens: log-rates 2.1e-2 of max|ref|, loss
5.5e-4, worst gradient 0.159 norm-relative = layer 0's attention-output weight, whose gradient sums
3,136 token outer products of fp8-derived activations and cancels strongly).  bench.py --dtype fp8
checks its full benched batch against the same bars (one definition, not two)."""

FP8_OUT = 4e-2     # log-rates, max abs error / max |ref|
FP8_LOSS = 2e-3    # loss, relative
FP8_GRAD = 3e-1    # gradients, norm-relative
