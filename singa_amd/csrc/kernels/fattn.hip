// Fused multi-head attention for the in-place [B][S][3][H][D] projection
// (BERT's QKVAttention, the sonnx-imported attention chain): one workgroup
// per (batch, head) does QK^T, the softmax and PV in registers and LDS -- the
// fp32 [B*H][S][S] score tensor, the separate softmax pass and the bf16
// probability tensor of the unfused path (ops/functional.py
// attention_qkv_fwd: two batched GEMMs + softmax) never exist.  The forward
// keeps only the per-row log-sum-exp; the backward recomputes P from it
// (flash-attention style) and writes dQ / dK / dV straight into their slots of
// d(qkv), optionally summing their columns into the q/k/v projection's bias
// gradient on the way (no separate column-sum pass over d(qkv)).
//
// Shapes: D = 64, S <= 128, S % 32 == 0 (host-checked; anything else takes
// the unfused path).  Additive key mask (BERT's [B][1][1][S] padding mask) or
// none.  Reference softmax surface: include/mshadow/cuda/tensor_gpu-inl.cuh:172-228.
//
// MFMA layout (v_mfma_f32_16x16x32_bf16, D = A B): lane l = 16 g + i holds
// A[i][8g..8g+7], B[8g..8g+7][i] and D[4g..4g+3][i].  QK^T runs as K Q^T so
// each lane owns ONE query row (i) and four keys per 16-key block: the row max
// and sum are in-lane plus two cross-lane steps, and the probabilities are
// already the A operand of PV -- the contraction order of a 32-key chunk is
// permuted (slot 8g+t <-> key 4g+t of the chunk's first block, slot 8g+4+t <->
// key 4g+t of its second), and V's B operand is fetched in that order with
// ds_read_b64_tr_b16 from a row-major [key][d] image.  The backward uses the
// same trick for dV += P^T dO and dK += dS^T Q, and stages dS in LDS for
// dQ = dS K.
#include "common.h"

namespace sg {
namespace fa {

constexpr int D = 64;
constexpr int SMAX = 128;
constexpr int NW = 8;     // waves per workgroup (one 16-row block each at S = 128)
constexpr int RS = 144;  // LDS row stride of a [S][64] bf16 image: 128 B + 16 (conflict-free 16-B and tr reads)

struct Args {
  const bf16* qkv;      // [B][S][3][H][D]
  int S, H;
  int64_t E;            // token row stride of qkv (3 H D)
  bf16* o;              // forward output [B][S][H D]
  int64_t ldo;          // H D
  float* lse;           // [B H][S]
  const float* mask;    // additive key mask mask[b * mstride + key], or null
  int64_t mstride;
  float scale;
  const bf16* dout;     // backward: dO, laid out like o
  const bf16* out;      // backward: the forward output O
  bf16* dqkv;           // backward: d(qkv), laid out like qkv
  float* dbias;         // backward: += column sums of d(qkv) over all B S rows (the q/k/v projection's bias
                        // gradient, fp32 [3][H][D]), or null
};

// Staging of NI [S][64] bf16 matrices into LDS images: every thread issues
// ALL its 16-byte global loads first (vector e = row e >> 3, chunk e & 7;
// VPI per image at S = SMAX), then writes them.  The loads are unconditional
// (rows past S re-read row 0 and are not stored): a load inside a divergent
// branch gets an s_waitcnt vmcnt(0) at the branch join, which serialised the
// first version's loads (one global latency each).
constexpr int VPI = SMAX * 8 / (64 * NW);

template <int NI>
__device__ __forceinline__ void stage(char* const (&img)[NI], const bf16* const (&src)[NI],
                                      const int64_t (&ld)[NI], int S, uint4 (&x)[NI][VPI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int v = 0; v < VPI; ++v) {
      int e = threadIdx.x + v * 64 * NW;
      e = e < S * 8 ? e : 0;
      x[i][v] = *(const uint4*)(src[i] + (e >> 3) * ld[i] + (e & 7) * 8);
    }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int v = 0; v < VPI; ++v) {
      const int e = threadIdx.x + v * 64 * NW;
      if (e < S * 8) *(uint4*)(img[i] + (e >> 3) * RS + (e & 7) * 16) = x[i][v];
    }
}

// row-major fragment: lane (g, i) -> row r0 + i, k = 32 kk + 8 g .. + 7 (A or B operand)
__device__ __forceinline__ bf16x8 frag_rm(const char* img, int stride, int r0, int kcol) {
  const int l = threadIdx.x & 63;
  return *(const bf16x8*)(img + (r0 + (l & 15)) * stride + (kcol + 8 * (l >> 4)) * 2);
}

// transposed fragment (B operand, k = rows of a row-major image): lane (g, i)
// gets B[slot 8g + t][col c0 + i] = img[R0 + t][c0 + i] (t < 4) and
// img[R1 + t - 4][c0 + i] (t >= 4); R0 / R1 are this lane group's row bases
__device__ __forceinline__ bf16x8 frag_tr(const char* img, int R0, int R1, int c0) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  const int i = threadIdx.x & 15;
  const int col = (c0 + 4 * (i & 3)) * 2;
  const v4s x0 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + (R0 + (i >> 2)) * RS + col));
  const v4s x1 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + (R1 + (i >> 2)) * RS + col));
  i16x8 r;
  r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
  r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A wave's 16 x 64 output block (MFMA layout: lane (g, i) holds rows 4g + j,
// column 16 db + i) -> global rows dst + r * ld, through the wave's own LDS
// scratch (16 rows of OS bytes): 16-byte stores of 8 consecutive columns
// instead of 2-byte ones.
constexpr int OS = 64 * 2 + 16;  // scratch row stride (bytes)
constexpr int WSCR = 16 * OS;    // per-wave scratch
__device__ __forceinline__ void store_block(char* scr, const f32x4 (&acc)[4], float scale, bf16* dst, int64_t ld) {
  const int l = threadIdx.x & 63, g = l >> 4, li = l & 15;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int j = 0; j < 4; ++j) *(bf16*)(scr + (4 * g + j) * OS + (db * 16 + li) * 2) = (bf16)(acc[db][j] * scale);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's scratch writes done
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int e = l + 64 * v, r = e >> 3, c = e & 7;
    *(uint4*)(dst + r * ld + c * 8) = *(const uint4*)(scr + r * OS + c * 16);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // reads done before the scratch is reused
  __builtin_amdgcn_wave_barrier();
}

// column sums of a wave's stored 16 x 64 block (the bf16 values store_block
// writes) into per-lane partials: lane (g, i) adds its rows 4g..4g+3 of
// column 16 db + i
__device__ __forceinline__ void colsum_block(const f32x4 (&acc)[4], float scale, float (&cs)[4]) {
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int j = 0; j < 4; ++j) cs[db] += (float)(bf16)(acc[db][j] * scale);
}

// grid B*H, 64 NW threads; LDS 3 S RS
__global__ void __launch_bounds__(64 * NW) fwd_k(const Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int S = a.S, H = a.H;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  char* sQ = smem;
  char* sK = smem + S * RS;
  char* sV = sK + S * RS;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, g = l >> 4, li = l & 15;
  char* scr = sV + S * RS + w * WSCR;
  const bf16* base = a.qkv + (int64_t)b * S * a.E + h * D;
  const int nkb = S / 16;
  const float* mrow = a.mask ? a.mask + (int64_t)b * a.mstride : nullptr;
  // this lane's key-mask values (keys kb*16 + 4g + j), loaded with the staging
  f32x4 mks[SMAX / 16];
#pragma unroll
  for (int kb = 0; kb < SMAX / 16; ++kb) mks[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (mrow) {
#pragma unroll
    for (int kb = 0; kb < SMAX / 16; ++kb) mks[kb] = *(const f32x4*)(mrow + (kb < nkb ? kb : 0) * 16 + 4 * g);
  }
  {
    uint4 x[3][VPI];
    char* const img[3] = {sQ, sK, sV};
    const bf16* const src[3] = {base, base + H * D, base + 2 * H * D};
    const int64_t ld[3] = {a.E, a.E, a.E};
    stage<3>(img, src, ld, S, x);
  }
  __syncthreads();
  for (int qb = w; qb < nkb; qb += NW) {
    const int q0 = qb * 16;
    const bf16x8 fq0 = frag_rm(sQ, RS, q0, 0), fq1 = frag_rm(sQ, RS, q0, 32);
    f32x4 s[SMAX / 16];
    float mx = -3.0e38f;
#pragma unroll
    for (int kb = 0; kb < SMAX / 16; ++kb) {
      if (kb < nkb) {
        f32x4 t = {0.f, 0.f, 0.f, 0.f};
        t = mfma(frag_rm(sK, RS, kb * 16, 0), fq0, t);   // D[key][query]: keys kb*16 + 4g + j, query q0 + li
        t = mfma(frag_rm(sK, RS, kb * 16, 32), fq1, t);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          t[j] = t[j] * a.scale + mks[kb][j];
          mx = fmaxf(mx, t[j]);
        }
        s[kb] = t;
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < SMAX / 16; ++kb) {
      if (kb < nkb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s[kb][j] = __expf(s[kb][j] - mx);
          sum += s[kb][j];
        }
      }
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.f / sum;
    if (g == 0) a.lse[(int64_t)bh * S + q0 + li] = mx + __logf(sum);
    f32x4 o[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < SMAX / 32; ++c) {
      if (c < nkb / 2) {
        bf16x8 pa;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = (bf16)(s[2 * c][j] * inv);
          pa[4 + j] = (bf16)(s[2 * c + 1][j] * inv);
        }
#pragma unroll
        for (int db = 0; db < 4; ++db)
          o[db] = mfma(pa, frag_tr(sV, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), o[db]);  // D[query][d]
      }
    }
    store_block(scr, o, 1.f, a.o + ((int64_t)b * S + q0) * a.ldo + h * D, a.ldo);
  }
}

// grid B*H, 64 NW threads; LDS 4 S RS + S (2S + 16) + 8 S + NW WSCR (+ NW * 4 * 3 * 64 floats with dbias)
__global__ void __launch_bounds__(64 * NW) bwd_k(const Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int S = a.S, H = a.H;
  const int SS = 2 * S + 16;  // dS image row stride (bytes)
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  char* sQ = smem;
  char* sK = sQ + S * RS;
  char* sV = sK + S * RS;
  char* sO = sV + S * RS;  // dO
  char* sdS = sO + S * RS;
  float* sL = (float*)(sdS + S * SS);
  float* sD = sL + S;
  char* scr_base = (char*)(sD + S);
  float* sCS = (float*)(scr_base + NW * WSCR);  // [NW][4][q, k, v][64] partial column sums of this (b, h)
  const bf16* base = a.qkv + (int64_t)b * S * a.E + h * D;
  {
    // one image at a time: measured faster here than stage() with all four
    // images' loads in flight (25.7 vs 31-33 us per BERT-base layer,
    // profiles/r6/attention_staging_ab.txt) -- unlike the forward (9.7 vs 15 us)
    const bf16* const srcs[4] = {base, base + H * D, base + 2 * H * D, a.dout + (int64_t)b * S * a.ldo + h * D};
    char* const imgs[4] = {sQ, sK, sV, sO};
    const int64_t lds_[4] = {a.E, a.E, a.E, a.ldo};
    for (int i = 0; i < 4; ++i)
      for (int v = threadIdx.x; v < S * 8; v += blockDim.x) {
        const int r = v >> 3, c = v & 7;
        *(uint4*)(imgs[i] + r * RS + c * 16) = *(const uint4*)(srcs[i] + r * lds_[i] + c * 8);
      }
    for (int q = threadIdx.x; q < S; q += blockDim.x) sL[q] = a.lse[(int64_t)bh * S + q];
  }
  // Delta[q] = sum_d dO[q][d] O[q][d] (four threads per row, 16 d each)
  {
    const int t = threadIdx.x;
    float acc = 0.f;
    const int q = t >> 2, hf = t & 3;
    {
      const int qq = q < S ? q : 0;  // (unconditional loads: no vmcnt(0) per branch join)
      const bf16* orow = a.out + ((int64_t)b * S + qq) * a.ldo + h * D + hf * 16;
      const bf16* drow = a.dout + ((int64_t)b * S + qq) * a.ldo + h * D + hf * 16;
      bf16x8 x[2], y[2];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        x[v] = *(const bf16x8*)(orow + v * 8);
        y[v] = *(const bf16x8*)(drow + v * 8);
      }
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += (float)x[v][j] * (float)y[v][j];
      if (q >= S) acc = 0.f;
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (q < S && hf == 0) sD[q] = acc;
  }
  __syncthreads();
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, g = l >> 4, li = l & 15;
  const int nkb = S / 16;
  const float* mrow = a.mask ? a.mask + (int64_t)b * a.mstride : nullptr;
  const int64_t E = a.E;
  float csq[4] = {0.f, 0.f, 0.f, 0.f}, csk[4] = {0.f, 0.f, 0.f, 0.f}, csv[4] = {0.f, 0.f, 0.f, 0.f};
  // phase 1: dK, dV of key blocks kb = w, w + NW, ...; dS into LDS
  for (int kb = w; kb < nkb; kb += NW) {
    const int k0 = kb * 16;
    const float mk = mrow ? mrow[k0 + li] : 0.f;
    const bf16x8 fk0 = frag_rm(sK, RS, k0, 0), fk1 = frag_rm(sK, RS, k0, 32);
    const bf16x8 fv0 = frag_rm(sV, RS, k0, 0), fv1 = frag_rm(sV, RS, k0, 32);
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      dv[db] = f32x4{0.f, 0.f, 0.f, 0.f};
      dk[db] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int c = 0; c < nkb / 2; ++c) {
      bf16x8 pa, dsa;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q0 = (2 * c + u) * 16;
        f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        st = mfma(frag_rm(sQ, RS, q0, 0), fk0, st);  // D[query][key]: queries q0 + 4g + j, key k0 + li
        st = mfma(frag_rm(sQ, RS, q0, 32), fk1, st);
        dp = mfma(frag_rm(sO, RS, q0, 0), fv0, dp);  // dP[query][key]
        dp = mfma(frag_rm(sO, RS, q0, 32), fv1, dp);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + 4 * g + j;
          const float p = __expf(st[j] * a.scale + mk - sL[q]);
          const float ds = p * (dp[j] - sD[q]);
          pa[4 * u + j] = (bf16)p;
          const bf16 dsb = (bf16)ds;
          dsa[4 * u + j] = dsb;
          *(bf16*)(sdS + q * SS + (k0 + li) * 2) = dsb;
        }
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        // dV[key][d] += sum_q P[q][key] dO[q][d];  dK[key][d] += sum_q dS[q][key] Q[q][d]
        dv[db] = mfma(pa, frag_tr(sO, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), dv[db]);
        dk[db] = mfma(dsa, frag_tr(sQ, 32 * c + 4 * g, 32 * c + 16 + 4 * g, db * 16), dk[db]);
      }
    }
    // D[key][d]: keys k0 + 4g + j, d = db*16 + li
    bf16* krow = a.dqkv + ((int64_t)b * S + k0) * E + H * D + h * D;
    store_block(scr_base + w * WSCR, dk, a.scale, krow, E);
    store_block(scr_base + w * WSCR, dv, 1.f, krow + H * D, E);
    if (a.dbias) {
      colsum_block(dk, a.scale, csk);
      colsum_block(dv, 1.f, csv);
    }
  }
  __syncthreads();  // dS complete
  // phase 2: dQ of query blocks qb = w, w + NW, ...: dQ = scale dS K
  for (int qb = w; qb < nkb; qb += NW) {
    const int q0 = qb * 16;
    f32x4 dq[4];
#pragma unroll
    for (int db = 0; db < 4; ++db) dq[db] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nkb / 2; ++c) {
      const bf16x8 fa = frag_rm(sdS, SS, q0, 32 * c);  // dS[query][keys 32c + 8g ..]
#pragma unroll
      for (int db = 0; db < 4; ++db)
        dq[db] = mfma(fa, frag_tr(sK, 32 * c + 8 * g, 32 * c + 8 * g + 4, db * 16), dq[db]);
    }
    store_block(scr_base + w * WSCR, dq, a.scale, a.dqkv + ((int64_t)b * S + q0) * E + h * D, E);
    if (a.dbias) colsum_block(dq, a.scale, csq);
  }
  if (a.dbias) {  // (uniform branch)
    // every lane stores its 12 partial column sums into its own slot of an
    // [NW][4][3 D] LDS image (plain stores, conflict-free), then 3 D threads
    // each fold 4 NW slots and issue one global atomic.  (LDS float atomics
    // from the lanes cost 5-16 us per launch here; shuffles + LDS atomics ~5.)
    float* slot = sCS + (w * 4 + g) * 3 * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      slot[db * 16 + li] = csq[db];
      slot[D + db * 16 + li] = csk[db];
      slot[2 * D + db * 16 + li] = csv[db];
    }
    // raw barrier after the LDS stores only: __syncthreads' fence would first
    // wait for this wave's dQ / dK / dV global stores
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x < 3 * D) {
      const int part = threadIdx.x / D, c = threadIdx.x - part * D;
      float v = 0.f;
#pragma unroll 8
      for (int k = 0; k < 4 * NW; ++k) v += sCS[k * 3 * D + threadIdx.x];
      atomicAdd(a.dbias + (int64_t)part * H * D + h * D + c, v);
    }
  }
}

}  // namespace fa
}  // namespace sg

using sg::fa::Args;

static bool fattn_ok(int S, int D) { return D == sg::fa::D && S >= 32 && S <= sg::fa::SMAX && S % 32 == 0; }

extern "C" int sg_fattn_ok(int S, int D) { return fattn_ok(S, D) ? 1 : 0; }

extern "C" int sg_fattn_fwd(const void* qkv, void* o, float* lse, const float* mask, int64_t mstride, int B, int S,
                            int H, int D, float scale, hipStream_t s) {
  if (!fattn_ok(S, D) || B <= 0 || H <= 0) return -1;
  Args a{};
  a.qkv = (const sg::bf16*)qkv;
  a.S = S;
  a.H = H;
  a.E = 3LL * H * D;
  a.o = (sg::bf16*)o;
  a.ldo = (int64_t)H * D;
  a.lse = lse;
  a.mask = mask;
  a.mstride = mstride;
  a.scale = scale;
  const int lds = 3 * S * sg::fa::RS + sg::fa::NW * sg::fa::WSCR;
  hipLaunchKernelGGL(sg::fa::fwd_k, dim3(B * H), dim3(64 * sg::fa::NW), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int sg_fattn_bwd(const void* qkv, const void* o, const void* dout, const float* lse, const float* mask,
                            int64_t mstride, void* dqkv, float* dbias, int B, int S, int H, int D, float scale,
                            hipStream_t s) {
  if (!fattn_ok(S, D) || B <= 0 || H <= 0) return -1;
  Args a{};
  a.qkv = (const sg::bf16*)qkv;
  a.S = S;
  a.H = H;
  a.E = 3LL * H * D;
  a.ldo = (int64_t)H * D;
  a.lse = (float*)lse;
  a.mask = mask;
  a.mstride = mstride;
  a.scale = scale;
  a.dout = (const sg::bf16*)dout;
  a.out = (const sg::bf16*)o;
  a.dqkv = (sg::bf16*)dqkv;
  a.dbias = dbias;
  const int cs = sg::fa::NW * 4 * 3 * sg::fa::D * (int)sizeof(float);  // partial column-sum slots
  const int lds = 4 * S * sg::fa::RS + S * (2 * S + 16) + 8 * S + sg::fa::NW * sg::fa::WSCR + (dbias ? cs : 0);
  static bool attr = hipFuncSetAttribute((const void*)sg::fa::bwd_k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         4 * sg::fa::SMAX * sg::fa::RS + sg::fa::SMAX * (2 * sg::fa::SMAX + 16) +
                                             8 * sg::fa::SMAX + sg::fa::NW * sg::fa::WSCR + cs) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL(sg::fa::bwd_k, dim3(B * H), dim3(64 * sg::fa::NW), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
