// gemm_dw.h — the token-reduction weight-gradient GEMM (gemm_dw.hip), used by vs_gemm.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "vspike.h"

namespace vs {

struct DwGrid {
  int tiles_m, tiles_n, splits, ksteps;  // ksteps: 64-token steps per split
};

struct DwPlan {
  bool valid, swap;  // swap: the kernel runs on (B, A) and stores C transposed
  int BM, BN;        // output tile: BM (64, 128, 192) rows of the narrow operand x BN (64, 128) columns
  int stages;        // LDS-DMA ring depth (3 or 4)
  DwGrid g;
  int64_t part_floats, sum_floats;
};

// the patch embedding's weight gradient with the tubelet gather in the B-operand load (no cols):
// pixels f32 (B, F, C, H, W), tubelet 2, patch 16; token m = (b, f', hp, wp), column k = (c, t, i, j)
struct PatchDwGeo {
  int F, C, H, W;
  int n_tok, HpWp, Wp;
  float inv_ntok, inv_hpwp, inv_wp;  // float reciprocals (token index < 2^24, corrected by one step)
};

DwPlan plan_dw(int64_t M, int64_t N, int64_t K);
size_t dw_workspace_bytes(int64_t M, int64_t N, int64_t K);
int launch_dw(const vs_gemm_desc* d, hipStream_t s);
// dW[D][K] += dx^T gather(px), db[D] += column sums of dx (bf16 dx [tokens][lddx]); the plan of
// dw_workspace_bytes(D, K, tokens)
int launch_patch_dw(const bf16_t* dx, int64_t lddx, int64_t D, const float* px, const PatchDwGeo& g, int64_t tokens,
                    int64_t K, float* dw, int64_t ldw, float* db, float* ws, hipStream_t s);

// skinny split-K (M <= 64, N <= 256, both operands K-contiguous, bf16 or f32): partials [splits][M][N] in the workspace
bool skinny_ok(const vs_gemm_desc* d);
size_t skinny_workspace_bytes(int32_t dtype, int64_t M, int64_t N, int64_t K);
int launch_skinny(const vs_gemm_desc* d, hipStream_t s, int* splits_out);

}  // namespace vs
