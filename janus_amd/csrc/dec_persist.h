// Persistent decoder segments (dec_persist.hip): the launches between a layer's self- and
// cross-attention (segment A) and between its cross-attention and the next layer's
// self-attention (segment B) as resident grids with in-launch barriers.
#pragma once
#include "common.h"

namespace janus {

struct DecSegArgs {
  int B, MT;                 // rows (<= 256), 16-row tiles (power of two >= B / 16)
  float* x;                  // [B][512] fp32 residual stream (read-modify-write)
  // segment A: x += o Wo^T + bo; xqk = LN2(x) Wqk^T + bqk
  const _Float16* o; const _Float16* wo; const float* bo;
  const float* ln2g; const float* ln2b;
  const _Float16* wqk; const float* bqk; _Float16* xqk;     // xqk [B][8 * 512]
  // segment B: o' = c_h Wv_h^T + bv; x += o' Wo_c^T + bo_c; f = gelu(LN3(x) W1^T + b1);
  // x += f W2^T + b2; [wqkv != null] q, K/V = LN1'(x) Wqkv'^T + bqkv'
  const _Float16* xc;                                        // [B][8 * 512] (cross-attention)
  const _Float16* wv; const float* bv; _Float16* omid;       // omid [B][512] scratch
  const _Float16* woc; const float* boc;
  const float* ln3g; const float* ln3b;
  const _Float16* w1; const float* b1; _Float16* f;          // f [B][2048] scratch
  const _Float16* w2; const float* b2;
  const float* ln1g; const float* ln1b;                      // the NEXT layer's
  const _Float16* wqkv; const float* bqkv; _Float16* qkv;    // qkv [B][1536] (q part)
  _Float16* kc; _Float16* vc; int pos, n_ctx; const int32_t* roff;  // the next layer's cache
  unsigned* bar;             // 160 zeroed words (barrier counters, self-cleaning)
  unsigned* err;             // timeout flag (host-checked)
  long long* prof;           // phase stamps (JANUS_PHASE_PROF builds, tools/seg_prof.py); null
  // [wqkv == null, fin_out != null] the last layer's segment B ends with the decoder's final
  // LayerNorm of x -> fin_out [B][512] fp16 (layernorm_kernel's arithmetic), read by the
  // vocabulary projection: no LayerNorm launch
  const float* fing; const float* finb; _Float16* fin_out;
  // [enc != null] the layer / head kernel ends with the cross-attention of the layer whose
  // segment A it ran (xattn_body, one key split: xqk -> xc), as a phase after a barrier
  const _Float16* enc; int Te;                               // enc [B][Te][512]
};

// The layer kernel's segment A runs the NEXT layer's weights over the same buffers: only
// these change against segment B's DecSegArgs (its qkv / kc / vc / pos / roff / o feed the
// self-attention phase between them, 64-wide heads, scale 1/8).
struct DecSegNext {
  const _Float16* wo; const float* bo;
  const float* ln2g; const float* ln2b;
  const _Float16* wqk; const float* bqk;
};

// 16-row tiles for B rows (0: unsupported, B > 256)
int dec_seg_mtiles(int B);
// blocks of the resident grid on a partition of `cus` CUs (0: unsupported); 256 rows run
// one block per CU taking two blocks' work, or with `two_per_cu` two blocks per CU
int dec_seg_grid(int B, int cus, bool two_per_cu = false);
bool dec_seg_supported(int d, int H, int B, int cus);
// the resident grid fits: blocks per CU (occupancy of the segment kernels with their LDS)
// times the partition's CUs cover `grid`
bool dec_seg_resident(int grid, int cus);
void dec_seg_a_launch(const DecSegArgs& a, int grid, hipStream_t s);
void dec_seg_b_launch(const DecSegArgs& a, int grid, hipStream_t s);
// segment B of layer l (b: its args, with layer l + 1's QKV weights and cache), the
// self-attention of l + 1 and segment A of l + 1 (nx: its weights) in one launch
void dec_layer_launch(const DecSegArgs& b, const DecSegNext& nx, int grid, hipStream_t s);
// layer 0's head (g: segment A args of layer 0, with layer 0's LN1 / QKV weights and
// cache in ln1g / ln1b / wqkv / bqkv / kc / vc): q, K/V[pos] = LN1(x) Wqkv^T + bqkv, the
// self-attention and segment A of layer 0 in one launch (the QKV projection, self-attention
// and segment A launches before the first cross-attention)
void dec_head_launch(const DecSegArgs& g, int grid, hipStream_t s);
// JANUS_PHASE_PROF builds: the stamp buffer for layer l when JANUS_SEG_PROF=l, else null
long long* dec_seg_prof_target(int l);

}  // namespace janus
