// Persistent 3x3 / stride-1 / pad-1 convolution for the 64-channel, 56-wide
// ResNet-50 stage-1 shape (each bottleneck's conv2: x [N][56][56][64] ->
// y [N][56][56][64], bf16 NHWC), forward and data gradient.
//
// The reference computes it as per-image im2col + sgemm (ConvolutionLayer,
// src/worker/layer.cc:75-81 forward, :99-116 backward).  Through the generic
// implicit-GEMM kernel (igemm.hip) this shape runs at ~0.5 ms for 0.24 TFLOP
// and 0.82 GB: every 128 x 64 output tile re-gathers its 9 taps of input
// (9x the input bytes through L2), re-fetches the 72 KB filter bank and pays
// a prologue / epilogue for only nine K-tiles.
//
// Here one 512-thread workgroup per CU keeps the whole filter bank (64 x 576
// bf16, 72 KB) resident in LDS and walks a contiguous range of 8-output-row
// units (taken from a dynamic queue, common.h, so a workgroup that starts
// late -- its CU busy with communication kernels -- takes fewer).  Per unit the 10 input rows it needs (with a zero halo: the padding)
// are staged once into LDS, the next unit's rows already in flight in
// registers while this unit's 252 MFMAs per wave run.  Both LDS images are
// PLANAR by 16-byte channel chunk ([chunk][pixel] / [chunk][filter]): the 16
// lanes of an MFMA fragment read 16 consecutive pixels (or filters) of one
// chunk, which lands on 16 distinct bank quads for ANY pixel offset -- the
// tap shifts of a 3x3 window would break the usual row-XOR swizzle.  Fragment
// addresses are a per-lane base plus a compile-time immediate per (tap, half),
// so the K loop has no address arithmetic.
//
// Waves: 4 (pixel quarter: 7 blocks of 16 of the unit's 448 pixels) x 2
// (filter half: 32).  Epilogue per unit: bf16 NHWC stores plus, in registers
// across the whole range, the fused BatchNorm statistics of the output
// (forward: sum, sum of squares -- igemm's 32 atomic slot rows) or the
// identity-sum BN backward's masked gradient sum (data gradient: sum of the
// output where the producer BN's 1-bit ReLU mask is set; igemm stats_mode 3).
//
// Data gradient = the same convolution over dy with the filters flipped and
// transposed: W'[c][r'][s'][k] = W[k][2-r'][2-s'][c], read from the K-major
// copy WT [3][3][C][K] the dgrad path keeps (pretranspose_conv_weights).
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace sg {
namespace c3 {

template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

constexpr int CH = 64;                 // input channels = filters
constexpr int WD = 56;                 // width (input = output)
constexpr int PWD = WD + 2;            // patch row with the zero halo
constexpr int RB = 8;                  // output rows per unit
constexpr int PRW = RB + 2;            // patch rows
constexpr int NPIX = PRW * PWD;        // 580 patch pixels (halo columns included)
constexpr int NSLOT = PRW * WD * 8;    // fill slots: the 560 interior pixels x 8 chunks (the halo columns are
                                       // zeroed once and never written)
constexpr int PJ = 592 * 16;           // bytes of one chunk plane of the patch (592 = 16-multiple >= 584)
constexpr int PATCH = 8 * PJ;          // 75,776 B
constexpr int WJ = CH * 16;            // bytes of one chunk plane of the filters (64 filters x 16 B)
constexpr int WBYTES = 72 * WJ;        // 73,728 B: 9 taps x 8 chunks
constexpr int LDS = WBYTES + PATCH;    // 149,504 B
constexpr int NT = 512;
constexpr int PFH = (NSLOT / 2 + NT - 1) / NT;  // 5 staged 16-byte vectors per thread (one channel half)
constexpr int TMW = 7;                 // pixel blocks per wave: 448 / 16 / 4

struct Args {
  const bf16* x;         // [N][H][56][64]: x (forward) or dy (data gradient)
  const bf16* w;         // forward: W [64][3][3][64]; data gradient: WT [3][3][64][64]
  bf16* y;               // [N][H][56][64]
  float* stats;          // [32][2][64] slot rows (zeroed by the caller) or null
  const uint8_t* mask;   // data gradient: the producer BN's ReLU bits [N*H*56][8] (stats then = masked sum)
  int N, H;
  int units;             // N * H / 8
  int dbg;               // timing experiments only (SG_C3_DBG): bit 0 no output stores
  int* wq;               // dynamic unit queue slot (common.h) or null: static blockIdx partition
};

template <int WMODE>  // 0 forward, 1 data gradient
__global__ void __launch_bounds__(NT, 1) conv3x3_k(const Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x;
  const int ln = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;  // pixel quarter, filter half
  const int g4 = ln >> 4;

  // this workgroup's units: U0 = bx, U1 = bx + G, then (with a queue) U_i =
  // 2G + ticket, each ticket taken one unit ahead; (without) U_i = bx + i G
  const int G = (int)gridDim.x;
  int u = (int)blockIdx.x, un = u + G;
  int* sQ = (int*)(smem + LDS);  // ticket broadcast
  const int upi = a.H / RB;  // units per image

  // filter bank -> LDS plane [tap*8 + chunk][filter]; lanes take consecutive
  // filters so every wave-store is 1 KB contiguous
  for (int e = t; e < CH * 72; e += NT) {
    const int f = e & 63, jk = e >> 6;
    const int tap = jk >> 3, kc = jk & 7;
    const bf16* src = WMODE == 0 ? a.w + f * 576 + tap * 64 + kc * 8 : a.w + ((8 - tap) * 64 + f) * 64 + kc * 8;
    *(uint4*)(smem + jk * WJ + f * 16) = *(const uint4*)src;
  }

  // halo columns (patch columns 0 and 57 of every row): zero for good
  for (int e = t; e < 8 * PRW * 2; e += NT) {
    const int j = e / (PRW * 2), rr = (e >> 1) % PRW, side = e & 1;
    *(uint4*)(smem + WBYTES + j * PJ + (rr * PWD + side * (PWD - 1)) * 16) = make_uint4(0, 0, 0, 0);
  }

  // The patch is refilled one channel HALF at a time: the k-steps run all
  // taps of channels 0-31 (planes 0-3) first, then all taps of channels 32-63
  // (planes 4-7), so each half's planes are dead while the other half
  // computes and take the next data then -- no stall at a unit boundary.
  // Fill slot e of a half: interior pixel P' = 16 (e >> 6) + (e & 15) of the
  // unit's 10 input rows (contiguous in memory: row pr = P' / 56 starts at
  // input row ih0 + pr), chunk j = (e >> 4) & 3 of the half -- a wave reads
  // 16 pixels x 64 B and each 8-lane store group writes 8 consecutive pixels
  // of one plane.  Slot k of thread t is slot 0 plus 128 pixels.
  const int P0 = (t >> 6) * 16 + (t & 15), j0 = (t >> 4) & 3;
  uint4 v[PFH];
  auto load_half = [&](int u, int h) {
    const int n = u / upi, hg = u - n * upi;
    const bf16* src = a.x + ((int64_t)n * a.H + hg * RB - 1) * WD * CH + P0 * CH + (h * 4 + j0) * 8;
    const int plo = hg == 0 ? WD : 0;                                   // row -1 is padding
    const int phi = hg == upi - 1 ? (PRW - 1) * WD : PRW * WD;          // row H is padding
#pragma unroll
    for (int k = 0; k < PFH; ++k) {
      const int Pp = P0 + 128 * k;
      uint4 z = make_uint4(0, 0, 0, 0);
      if (Pp >= plo && Pp < phi) z = *(const uint4*)(src + k * 128 * CH);
      v[k] = z;
    }
  };
  auto store_half = [&](int h) {
#pragma unroll
    for (int k = 0; k < PFH; ++k) {
      const int Pp = P0 + 128 * k;
      const int pr = Pp / WD;
      if (Pp < PRW * WD) *(uint4*)(smem + WBYTES + (h * 4 + j0) * PJ + (Pp + 2 * pr + 1) * 16) = v[k];
    }
  };

  // per-lane fragment bases: A = pixel p = (wm*7 + i)*16 + (ln & 15) of the
  // unit (row p / 56, column p % 56; its tap (0, 0) sits at patch pixel
  // row*58 + column), chunk g4 (+4 for the upper half of a tap's channels);
  // B = filter wn*32 + (ln & 15) (+16 for jb = 1), chunk g4
  int abase[TMW];
#pragma unroll
  for (int i = 0; i < TMW; ++i) {
    const int p = (wm * TMW + i) * 16 + (ln & 15);
    const int orow = p / WD, ocol = p - orow * WD;
    abase[i] = WBYTES + g4 * PJ + (orow * PWD + ocol) * 16;
  }
  const int bbase = g4 * WJ + (wn * 32 + (ln & 15)) * 16;
  typedef const __attribute__((address_space(3))) char* lds_cp;
  const lds_cp L = (lds_cp)(__attribute__((address_space(3))) char*)smem;

  float s_sum[2][4], s_sq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_sum[j][r] = s_sq[j][r] = 0.f;

  // Epilogue of a finished unit, one pixel block i at a time: it runs inside
  // the NEXT unit's first-half MFMAs (acc_prev), so its stores and the
  // statistics' VALU fill the MFMA gaps instead of a phase of their own.
  f32x4 acc[TMW][2];
  bf16x4 accp[TMW][2];  // the finished unit, already rounded to the bf16 outputs
  unsigned mwp[TMW];
  auto epi = [&](int i, int64_t pix0) {
    const int64_t pix = pix0 + (wm * TMW + i) * 16 + (ln & 15);
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int f0 = wn * 32 + jb * 16 + 4 * g4;
      const bf16x4 o = accp[i][jb];
      if (!(a.dbg & 1)) *(bf16x4*)(a.y + pix * CH + f0) = o;
      if (a.stats) {
        if (WMODE == 1) {
          // the lane's two mask bytes (jb = 0, 1) sit in one aligned dword
          const unsigned mb = (mwp[i] >> (8 * (jb * 2 + (g4 >> 1)))) >> (f0 & 7);
#pragma unroll
          for (int r = 0; r < 4; ++r) s_sum[jb][r] += ((mb >> r) & 1u) != 0 ? (float)o[r] : 0.f;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float f = (float)o[r];
            s_sum[jb][r] += f;
            s_sq[jb][r] += f * f;
          }
        }
      }
    }
  };
  auto mask_loads = [&](int64_t pix0) {
    if (WMODE == 1 && a.stats) {
#pragma unroll
      for (int i = 0; i < TMW; ++i)
        mwp[i] = *(const unsigned*)(a.mask + (pix0 + (wm * TMW + i) * 16 + (ln & 15)) * 8 + wn * 4);
    }
  };

  // 9 k-steps (taps) of one channel half, software-pipelined by hand: the
  // next step's 9 fragments are read before this step's 14 MFMAs (left alone,
  // the compiler reused one fragment register and waited lgkmcnt(0) in front
  // of every MFMA pair).  EPI: run epilogue block i after the MFMAs of step i.
  bf16x8 fa[2][TMW], fb[2][2];
  auto frags = [&](auto khc, auto tapc, auto bc) {
    constexpr int kh = decltype(khc)::value, tap = decltype(tapc)::value, b = decltype(bc)::value;
    constexpr int dr = tap / 3, ds = tap % 3;
#pragma unroll
    for (int i = 0; i < TMW; ++i) fa[b][i] = *(const bf16x8*)(L + abase[i] + kh * 4 * PJ + (dr * PWD + ds) * 16);
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) fb[b][jb] = *(const bf16x8*)(L + bbase + (tap * 8 + kh * 4) * WJ + jb * 256);
  };
  auto half = [&](auto khc, bool epi_on, int64_t ppix0) {
    constexpr int kh = decltype(khc)::value;
    frags(khc, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    static_for<9>([&](auto tc) {
      constexpr int tap = decltype(tc)::value, b = tap & 1;
      if constexpr (tap + 1 < 9)
        frags(khc, std::integral_constant<int, tap + 1>{}, std::integral_constant<int, (tap + 1) & 1>{});
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
          acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b][jb], fa[b][i], acc[i][jb], 0, 0, 0);
      if constexpr (kh == 0 && tap < TMW) {
        if (epi_on) epi(tap, ppix0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  auto wait_lds_barrier = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's patch stores landed
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();        // raw: no drain of the output stores (vmcnt)
    asm volatile("" ::: "memory");
  };

  if (u < a.units) {
    load_half(u, 0);
    store_half(0);
    load_half(u, 1);
  }
  __syncthreads();  // the filters and the first unit's planes 0-3 are in
  bool have_prev = false;
  int64_t ppix0 = 0;
  while (u < a.units) {
    int ticket = 0;
    if (t == 0 && a.wq) ticket = wq_take(a.wq, 0);  // U_{i+2}
    // planes 0-3 hold this unit; every wave is done with planes 4-7
    store_half(1);
    if (un < a.units) load_half(un, 0);  // in flight during the first half
    if (have_prev) mask_loads(ppix0);
#pragma unroll
    for (int i = 0; i < TMW; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    half(std::integral_constant<int, 0>{}, have_prev, ppix0);
    wait_lds_barrier();  // planes 4-7 hold this unit; every wave is done with planes 0-3
    if (un < a.units) {
      store_half(0);
      load_half(un, 1);  // in flight during the second half
    }
    half(std::integral_constant<int, 1>{}, false, 0);
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) accp[i][jb][r] = (bf16)acc[i][jb][r];
    have_prev = true;
    ppix0 = (int64_t)u * RB * WD;  // the unit's first output pixel
    if (t == 0) *sQ = a.wq ? 2 * G + ticket : un + G;
    wait_lds_barrier();  // (every thread read the previous ticket before the middle barrier)
    const int unn = __builtin_amdgcn_readfirstlane(*sQ);
    u = un;
    un = unn;
  }
  if (a.wq && t == 0) wq_done(a.wq, 1);
  if (have_prev) {
    mask_loads(ppix0);
#pragma unroll
    for (int i = 0; i < TMW; ++i) epi(i, ppix0);
  }
  if (!a.stats) return;
  // reduce the 16 lanes of equal g4 and the 4 waves of equal wn through LDS,
  // then one atomic per (filter, sum) into slot row blockIdx.x % 32 (the data
  // gradient has only the first sum: its second half is never added)
  __syncthreads();
  float* red = (float*)(smem + WBYTES);  // [8 waves][64 lanes][16]
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(wid * 64 + ln) * 16 + j * 4 + r] = s_sum[j][r];
      red[(wid * 64 + ln) * 16 + 8 + j * 4 + r] = s_sq[j][r];
    }
  __syncthreads();
  if (t < (WMODE == 1 ? 1 : 2) * CH) {  // one thread per (filter, which sum)
    const int f = t & (CH - 1), q = t >> 6;
    const int wnf = f >> 5, j = (f >> 4) & 1, gg = (f >> 2) & 3, r = f & 3;
    float s = 0.f;
    for (int w4 = 0; w4 < 4; ++w4) {
      const int wv = w4 * 2 + wnf;
      for (int i = 0; i < 16; ++i) s += red[(wv * 64 + gg * 16 + i) * 16 + q * 8 + j * 4 + r];
    }
    atomicAdd(a.stats + (blockIdx.x & 31) * 2 * CH + q * CH + f, s);
  }
}

}  // namespace c3
}  // namespace sg

static int g_c3_on = 1;  // conv3x3_set: A/B switch

extern "C" {

void sg_conv3x3_set(int on) { g_c3_on = on; }
int sg_conv3x3_enabled() { return g_c3_on; }

// Returns 1 when the persistent kernel took the convolution, 0 otherwise (the
// caller runs the generic implicit GEMM).  Geometry: 3x3, stride 1, pad 1,
// dilation 1, 64 -> 64 channels, width 56, H % 8 == 0.  wmode 0: forward with
// w = W [64][3][3][64]; 1: data gradient with w = WT [3][3][64][64] (K-major
// copy), x = dy.  stats: 32 x 2 x 64 slot rows (zeroed by the caller) or null;
// mask (wmode 1 with stats): the producer BN's ReLU bits.
int sg_conv3x3_ok(int N, int H, int W, int C, int K) {
  using namespace sg::c3;
  return g_c3_on && C == CH && K == CH && W == WD && H > 0 && (H % RB) == 0 && N > 0 &&
         (int64_t)N * H * WD * CH < (1LL << 31);
}

int sg_conv3x3_64(const void* x, const void* w, int wmode, void* y, void* stats, const void* mask, int N, int H,
                  int W, int C, int K, hipStream_t s) {
  using namespace sg::c3;
  if (!sg_conv3x3_ok(N, H, W, C, K) || (wmode == 1 && stats && !mask)) return 0;
  static const int dbg = getenv("SG_C3_DBG") ? atoi(getenv("SG_C3_DBG")) : 0;
  Args a{(const sg::bf16*)x, (const sg::bf16*)w, (sg::bf16*)y, (float*)stats, (const uint8_t*)mask, N, H,
         N * (H / RB), dbg, sg_workq_slot()};
  const int cus = sg_cu_count();
  const int grid = a.units < cus ? a.units : cus;
  auto go = [&](auto kern) {
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           LDS + 16) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), LDS + 16, s, a);
  };
  if (wmode == 0) go(conv3x3_k<0>);
  else go(conv3x3_k<1>);
  return 1;
}

}  // extern "C"
