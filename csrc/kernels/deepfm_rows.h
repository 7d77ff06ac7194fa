// Parameter blocks shared by the DeepFM row-tile kernel and its host launcher.
#pragma once
#include "../common.h"
#include "optim.h"
#include "push.h"

namespace rocfm {

constexpr int kMaxHidden = 6;  // hidden MLP layers supported by the fused engine
constexpr int kRowTile = 16;   // rows per workgroup = one 16-row MFMA M tile
constexpr int kRowThreads = 512;  // 8 waves

// compute_dtype=fp8: pre-quantised fp8-e4m3 copies of the input layer's weights, written by every
// weight refresh (wgrad epilogue, dense apply) next to the bf16 swizzled copies, with ONE scale per
// tensor taken from the previous weights' max |w| (delayed scaling: the refresh cannot know the
// new weights' max before it has written them).  Step s's refresh quantises with amax[s & 1] and
// accumulates the max of the weights it writes into amax[(s + 1) & 1], which step s's row kernel
// zeroed; a host refresh (track = 0) presets both slots to the exact max.  inv_scale = amax / 448
// of the copies' current quantisation: the row kernel's de-scale.
constexpr float kFp8Max = 448.f;  // largest finite e4m3fn
struct Fp8W0 {
  uint8_t* f = nullptr;  // frag_swz(o, i, dims[0]) like WTs[0]
  uint8_t* b = nullptr;  // frag_swz(i, o, dims[1]) like Wbs[0]
  float* amax = nullptr;       // [2]
  float* inv_scale = nullptr;  // [1]
  int track = 0;
};

struct RowsLds {  // byte offsets into dynamic LDS (all multiples of 16)
  int ids, vals, wx, S, ylin, g, act[kMaxHidden + 1], dzA, dzB, f32, pos, amax;
  int q8, ldq;          // fp8: the input layer's forward A operand (h0) quantised once per tile in
                        // phase B, [16][ldq] e4m3 bytes
  int nxt, gr;          // dedup: int [16·F] next member of each lookup's group; f32 [16·F][Kp] gradient rows
  int bnr[kMaxHidden];  // batch_norm: f32 [16][dims[l+1]] post-ReLU values r of layer l (kept for backward)
  int bnst[kMaxHidden]; // batch_norm: f32 [2][dims[l+1]] batch mean, 1/sqrt(var + eps) of layer l
  int bndy, bntot;      // batch_norm backward scratch: f32 [16][max dim] dy, [2][max dim] column totals
  int lda[kMaxHidden + 1];  // bf16 row stride of each activation tile
  int ldz;                  // bf16 row stride of the dz ping-pong tiles
  int prm;                  // f32 block of small parameters staged at kernel start:
  int prm_bias[kMaxHidden], prm_wout, prm_bout, prm_fmb, prm_lab, prm_n;  // (float offsets within it)
  int total;
};

struct RowsParams {
  // inputs
  const int32_t* ids;   // [B][F]
  const float* vals;    // [B][F]
  const float* labels;  // [B]
  const float* emb;     // [V][Kp]: cols 0..K-1 = fm_v row, col K = fm_w, rest 0
  int tbl_bf16;         // 1: emb holds bf16 rows (common.h tbl_load4)
  const float* fm_bias;
  const float* w_out;  // [dims[nl]] f32 (deep_out/weights)
  const float* b_out;  // [1]
  const uint16_t* WT[kMaxHidden];  // layer l: [dims[l+1]][dims[l]] bf16 (forward B operand)
  const uint16_t* Wb[kMaxHidden];  // layer l: [dims[l]][dims[l+1]] bf16 (backward B operand)
  const uint16_t* WTs[kMaxHidden];  // frag_swz copies of WT / Wb (compile-time-shape kernels load these)
  const uint16_t* Wbs[kMaxHidden];
  const float* bias[kMaxHidden];   // layer l: [dims[l+1]]
  float keep[kMaxHidden];
  int dims[kMaxHidden + 1];  // dims[0] = round_up(F*K, 32); dims[l>0] = hidden width padded to 32
  int nl, F, K, Kp, B, Bp;   // B valid rows; Bp = padded rows = leading dim of actT/dzT
  uint32_t magicF;           // floor(2^32/F)+1 (set by the launcher)
  float inv_scale;           // dL/dy scale (1/B_local)
  int train, loss_type;      // loss_type 0 log_loss, 1 square_loss
  uint64_t seed;
  const int64_t* step;  // device global_step (dropout key)
  // outputs
  float* prob;       // [B]
  float* loss_rows;  // [B] (nullable)
  float* g_out;      // [Bp] dL/dy
  float* contrib;    // [B*F][Kp] per-lookup gradient rows (train)
  uint16_t* actT[kMaxHidden + 1];  // [dims[a]][Bp] bf16, a = 0..nl (train)
  uint16_t* dzT[kMaxHidden + 1];   // [dims[a]][Bp] bf16, a = 1..nl (train)
  RowsLds lds;
  unsigned long long* stamps;  // diagnostic (nullable)
  const int32_t* contrib_pos;  // nullable [B][F]: row of contrib receiving each lookup's gradient
                               // (its position in the sorted lookup order), else row·F + field
  int32_t* zero_word;          // nullable: set to 0 at kernel start (DP: the export's row counter)
  int fp8;                     // 1: the input layer's forward GEMM on fp8-e4m3 MFMA (per-row activation
                               // and per-column weight scales; compile-time-shape kernels only)
  int force_generic;           // 1: never use a compile-time-shape instantiation (tests)
  int ablate;                  // diagnostics only (results invalid): bit0 skip h0ᵀ stores, bit1 skip
                               // the FM loop, bit2 skip the phase-B weight prefetch
  // batch_norm=True (PS:241-244, 316-338): y = γ·(r − μ_B)/√(σ²_B + ε) + β after each hidden ReLU,
  // batch moments over ALL B rows (grid-wide reductions inside the launch; runtime-shape kernel).
  int bn;
  const float* bn_gamma[kMaxHidden];  // [dims[l+1]] (inside the flat dense buffer)
  const float* bn_beta[kMaxHidden];
  float* bn_mean[kMaxHidden];         // moving averages: updated by training, read by inference
  float* bn_var[kMaxHidden];
  float bn_decay, bn_eps;
  int bn_dmax;                        // max hidden dim (stride of the scratch below)
  float* bn_part;                     // [2·nl][gridDim][bn_dmax][2] per-workgroup partial moments
  float* bn_grad;                     // [nl][2][bn_dmax]: Σ dy·x̂ (d γ), Σ dy (d β) of the batch
  unsigned* bn_sync;                  // [2] grid-barrier arrival / exit counters (0 between launches)
  int* bn_error;                      // set if a grid barrier timed out (the host check raises)
  PushTarget push;                    // producer push (push.h): workgroup 0 signals "entered"
  PushTarget push2;                   // a second exchange pushed by this step (row-shard X3)
  PushTarget push3;                   // a third (owner-sharded DP: X5, pushed by the owner merge)
  int row_tile;                       // examples per workgroup: 16, 8 or 4 (0 = default; static shapes)
  // per-tile dedup (batch.h DedupParams): contrib_pos holds each lookup's compacted group index (c
  // for the group's first lookup, ~c for the others) and contrib_nxt the next lookup of its group;
  // phase F sums every group's gradient rows in LDS (lookup order) and writes ONE row per group
  int dedup;
  const int32_t* contrib_nxt;
  Fp8W0 w8;  // fp8 kernels: the pre-quantised input-layer weights (the kernel reads f, b, inv_scale
             // and, training, zeroes amax[(step + 1) & 1])
  // row-tile split (deepfm_rows.hip CtShape G): `split` workgroups per row tile (0 / 1 = off; 2 for
  // the training kernel of a wide input layer, bf16, no dedup — the launcher falls back to 1
  // otherwise).  xbuf: [Bp / 8][dims[1]][16] bf16 exchange of layer 0's outputs; xctr: [Bp / 8]
  // arrival counters, zeroed once at allocation and never reset; xerr: set if an exchange wait
  // timed out (the host check raises; the counters must then be zeroed again).
  int split;
  // write-through (sc1) stores of the kernel's large outputs, so that the launch leaves less dirty
  // L2 to write back at its end: bit 0 the per-lookup gradient rows (contrib), bit 1 h0ᵀ (actT[0])
  int wt;
  uint16_t* xbuf;
  unsigned* xctr;
  int* xerr;
};

struct WgradParams {
  const uint16_t* actT[kMaxHidden + 1];
  const uint16_t* dzT[kMaxHidden + 1];
  const float* g;  // [Bp] dL/dy
  int dims[kMaxHidden + 1];
  int nl, Bp;
  float* params;  // flat dense buffer
  float* grads;   // flat grad buffer (fuse_opt == 0)
  float* s0;
  float* s1;
  int offW[kMaxHidden], offb[kMaxHidden], off_wout, off_bout, off_fmb;
  uint16_t* WT[kMaxHidden];
  uint16_t* Wb[kMaxHidden];
  uint16_t* WTs[kMaxHidden];  // frag_swz copies (nullable): WT as [Dout][Din], Wb as [Din][Dout]
  uint16_t* Wbs[kMaxHidden];
  int tile_start[kMaxHidden + 1];  // prefix sums of 32 × (32·tw) tiles per layer
  int tw[kMaxHidden];              // output subtiles per tile (1, 2, 4; set by wgrad_prepare)
  int bias_start[kMaxHidden + 1];  // prefix sums of 32-column bias blocks per layer
  int fuse_opt;
  OptParams opt;
  const int64_t* step;
  float grad_scale;
  unsigned long long* stamps;  // diagnostic (nullable)
  int bn;                      // batch_norm: emit d γ / d β of every layer from bn_grad
  const float* bn_grad;        // [nl][2][bn_dmax] (written by deepfm_rows)
  int bn_dmax;
  int off_gamma[kMaxHidden], off_beta[kMaxHidden];
  PushTarget push;  // DP fused push (fuse_opt == 0): gradients go straight into the W receive slots
  int push_mirror;  // with push: also store every gradient locally (grads) — the shadow exchange
                    // all-gathers the local buffer and compares it with what the producers pushed
  Fp8W0 w8;         // fused optimizer: refresh the fp8 input-layer copies too (f == nullptr: none)
};

struct DenseApplyParams {
  float* params;
  const float* grads;
  float* s0;
  float* s1;
  int n;
  int nl;
  int dims[kMaxHidden + 1];
  int offW[kMaxHidden];
  uint16_t* WT[kMaxHidden];
  uint16_t* Wb[kMaxHidden];
  uint16_t* WTs[kMaxHidden];  // frag_swz copies (nullable)
  uint16_t* Wbs[kMaxHidden];
  int apply;
  OptParams opt;
  const int64_t* step;
  float grad_scale;
  int nseg;                // > 1: grads are nseg rank segments (DP all-gather), summed in rank order
  long long seg_stride;    // floats between segments
  Fp8W0 w8;                // refresh the fp8 input-layer copies too (f == nullptr: none)
};

}  // namespace rocfm
