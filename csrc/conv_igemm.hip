// Implicit-GEMM 3x3 / 1x1 convolution, NHWC bf16, MFMA 16x16x32 (gfx950).
//
// Replaces the cuDNN/MIOpen conv forward the reference reaches through torch eager
// (/root/reference/pkg/segmentation_model.py:31,34 -> nn.Conv2d(k=3, pad=1, bias=False)).
// The same kernel computes conv dgrad (dX = conv(dY, flip(W)^T)) with a pre-transposed weight.
//
// GEMM view: out[m = pixel][n = cout] = sum_k im2col(x)[m][k] * W[n][k], k = (tap, cin).
//   * Two input sources are concatenated along channels (torch.cat([skip, up]) in Up.forward,
//     segmentation_model.py:75) so the concat is never materialised.
//   * Output may be split at channel Cy1 into two destinations (dgrad of the concat input).
//   * Epilogue optionally emits per-channel (sum, sumsq) partials of the bf16-rounded output for
//     training-mode BatchNorm (one slab row per M tile, reduced by bn_finalize).
//
// Tiling: block = 4 waves (256 threads), block tile BM x BN with each wave owning 64x64; K step
// = 64 channels of one tap. Both operand tiles are staged global->LDS by LDS-DMA
// (buffer_load ... lds, 16 B/lane) in MFMA-fragment-major order: one 1 KiB wave-instruction = one
// 16x32 MFMA operand fragment, so every ds_read_b128 is lane-contiguous (bank-conflict free).
// Halo/zero padding comes from out-of-range buffer offsets (hardware returns 0).
// Double-buffered LDS with ONE raw s_barrier per K step: tile k+1's DMA is issued right after the
// barrier that retires tile k and lands under tile k's MFMAs.
#include "common.h"

struct ConvArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2;  // channels in each source (source 2 may be empty)
  int pitch1, pitch2;  // pixel pitch (elements)
  const u16* w;
  uint32_t wbytes;
  int ldw;  // weight row length (elements) = taps * Cin (padded)
  u16* y1;
  u16* y2;
  uint32_t ybytes1, ybytes2;
  int Cy1;  // channels going to y1 (rest to y2)
  int ypitch1, ypitch2;
  float* stats;  // [tilesM][2][Cout] partial (sum, sumsq) or nullptr
  int N, H, W, Cout, M;
  int taps;  // 9 (3x3) or 1 (1x1)
  int packed;  // 1: Cin == 8, K packs 8 taps per 64-wide K step
  int nks;  // number of K steps
  int cpt;  // 64-channel chunks per tap (generic mode)
  int tilesN;
};

// ROWMAJ=0: fragment-major LDS image (each DMA piece = one MFMA fragment: 16 rows x 64 B).
// ROWMAJ=1: row-major [rows][128 B] image, 16-B chunk XOR-swizzled by (row & 7) on the SOURCE
//           address; each DMA piece = 8 full 128-B lines (half the TA line lookups per byte), and
//           the fragment ds_read_b128s stay bank-conflict free (checked by simulation).
template <int BM, int BN, int ROWMAJ>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(const ConvArgs a) {
  constexpr int WAVES_M = BM / 64;
  constexpr int NPR = BM / 64;        // pixel rows per lane handled by this wave's DMA
  constexpr int FW_PER_WAVE = BN / 32;  // weight fragments DMA'd per wave per K step
  constexpr int P_BYTES = BM * 128, W_BYTES = BN * 128, BUF = P_BYTES + W_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;

  const uint32_t nwg = gridDim.x;
  const uint32_t lid = xcd_remap(blockIdx.x, nwg);
  const int tm = lid / a.tilesN, tn = lid % a.tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);

  // ---- per-lane pixel rows this wave stages ----
  constexpr int NROW = ROWMAJ ? BM / 32 : NPR;  // distinct pixel rows per lane
  int pm[NROW], ph[NROW], pw[NROW];
  bool pv[NROW];
#pragma unroll
  for (int r = 0; r < NROW; ++r) {
    const int row = ROWMAJ ? (wave * NROW + r) * 8 + (lane >> 3) : (wave * NPR + r) * 16 + (lane & 15);
    const int m = m0 + row;
    pv[r] = m < a.M;
    const int mm = pv[r] ? m : 0;
    const int hw = mm % (a.H * a.W);
    pm[r] = mm;
    ph[r] = hw / a.W;
    pw[r] = hw - ph[r] * a.W;
  }
  const int qlane = lane >> 4;  // 16-B chunk (of 4) within a 32-wide K half (fragment-major)
  const int gch = (lane & 7) ^ (lane >> 3);  // row-major: global 16-B chunk fetched by this lane

  // weight rows for this wave's DMA pieces
  constexpr int WPIECES = ROWMAJ ? BN / 32 : FW_PER_WAVE;
  uint32_t woff[WPIECES];
#pragma unroll
  for (int f = 0; f < WPIECES; ++f) {
    if (ROWMAJ) {
      const int n = n0 + (wave * WPIECES + f) * 8 + (lane >> 3);
      woff[f] = (uint32_t)(n * a.ldw + gch * 8) * 2u;
    } else {
      const int fw = wave * FW_PER_WAVE + f;  // fragment id in [0, BN/16*2)
      const int j = fw >> 1, hf = fw & 1;
      const int n = n0 + j * 16 + (lane & 15);
      woff[f] = (uint32_t)(n * a.ldw + (qlane + 4 * hf) * 8) * 2u;
    }
  }

  auto issue = [&](int ks, char* buf) {
    // --- pixel (im2col) operand ---
    if constexpr (ROWMAJ) {
      if (a.packed) {
        const int tap = ks * 8 + gch;
        const int dr = tap / 3 - 1, ds = tap % 3 - 1;
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          const int hh = ph[r] + dr, ww = pw[r] + ds;
          const bool ok = pv[r] & (tap < 9) & inb(hh, a.H) & inb(ww, a.W);
          const uint32_t off = ok ? (uint32_t)((pm[r] + dr * a.W + ds) * a.pitch1) * 2u : RDP_OOB;
          dma16(rx1, (lds_void*)(buf + (wave * NROW + r) * 1024), off);
        }
      } else {
        const int tap = ks / a.cpt;
        const int c0 = (ks - tap * a.cpt) * 64;
        const bool s2 = c0 >= a.C1;
        const int ch = (s2 ? c0 - a.C1 : c0) + gch * 8;
        const int pitch = s2 ? a.pitch2 : a.pitch1;
        const int dr = a.taps == 9 ? tap / 3 - 1 : 0;
        const int ds = a.taps == 9 ? tap % 3 - 1 : 0;
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          const int hh = ph[r] + dr, ww = pw[r] + ds;
          const bool ok = pv[r] & inb(hh, a.H) & inb(ww, a.W);
          const uint32_t off = ok ? (uint32_t)((pm[r] + dr * a.W + ds) * pitch + ch) * 2u : RDP_OOB;
          dma16(s2 ? rx2 : rx1, (lds_void*)(buf + (wave * NROW + r) * 1024), off);
        }
      }
    } else if (a.packed) {
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int tap = ks * 8 + qlane + 4 * hf;
          const int dr = tap / 3 - 1, ds = tap % 3 - 1;
          const int hh = ph[r] + dr, ww = pw[r] + ds;
          const bool ok = pv[r] & (tap < 9) & inb(hh, a.H) & inb(ww, a.W);
          const uint32_t off = ok ? (uint32_t)((pm[r] + dr * a.W + ds) * a.pitch1) * 2u : RDP_OOB;
          dma16(rx1, (lds_void*)(buf + ((wave * NPR + r) * 2 + hf) * 1024), off);
        }
      }
    } else {
      const int tap = ks / a.cpt;
      const int c0 = (ks - tap * a.cpt) * 64;
      const bool s2 = c0 >= a.C1;
      const int ch = s2 ? c0 - a.C1 : c0;
      const int pitch = s2 ? a.pitch2 : a.pitch1;
      const int dr = a.taps == 9 ? tap / 3 - 1 : 0;
      const int ds = a.taps == 9 ? tap % 3 - 1 : 0;
#pragma unroll
      for (int r = 0; r < NPR; ++r) {
        const int hh = ph[r] + dr, ww = pw[r] + ds;
        const bool ok = pv[r] & inb(hh, a.H) & inb(ww, a.W);
        const uint32_t base = (uint32_t)((pm[r] + dr * a.W + ds) * pitch + ch + qlane * 8) * 2u;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const uint32_t off = ok ? base + hf * 64u : RDP_OOB;
          dma16(s2 ? rx2 : rx1, (lds_void*)(buf + ((wave * NPR + r) * 2 + hf) * 1024), off);
        }
      }
    }
    // --- weight operand ---
    char* wbuf = buf + P_BYTES;
#pragma unroll
    for (int f = 0; f < WPIECES; ++f) {
      const int fw = wave * WPIECES + f;
      dma16(rw, (lds_void*)(wbuf + fw * 1024), woff[f] + (uint32_t)ks * 128u);
    }
  };

  // LDS byte offsets of this lane's fragment reads (k-half hf) relative to subtile 0
  int rdoff[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
    rdoff[hf] = ROWMAJ ? (lane & 15) * 128 + 16 * (((lane >> 4) + 4 * hf) ^ (lane & 7)) : hf * 1024 + lane * 16;
  constexpr int SUBSTRIDE = 2048;  // bytes per 16-row subtile (both layouts)

  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One barrier per K step: the barrier retires this stage's DMA (every wave waited vmcnt(0)) and
  // every wave's LDS reads of the previous stage (lgkmcnt(0)), so the next stage can be issued into
  // the other buffer right after it and lands under this stage's MFMAs.
  issue(0, smem);
  for (int ks = 0; ks < a.nks; ++ks) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (ks + 1 < a.nks) issue(ks + 1, smem + ((ks + 1) & 1) * BUF);
    const char* pb = smem + (ks & 1) * BUF;
    const char* wb = pb + P_BYTES;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = *(const bf16x8*)(wb + (wn * 4 + j) * SUBSTRIDE + rdoff[hf]);
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = *(const bf16x8*)(pb + (wm * 4 + i) * SUBSTRIDE + rdoff[hf]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- epilogue: acc[j][i][r] = out[m = m0 + wm*64 + 16i + (lane&15)][n = n0 + wn*64 + 16j + 4*(lane>>4) + r]
  const auto ry1 = make_rsrc(a.y1, a.ybytes1);
  const auto ry2 = make_rsrc(a.y2 ? a.y2 : a.y1, a.y2 ? a.ybytes2 : 0u);
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
    const bool d2 = n >= a.Cy1;
    const int nn = d2 ? n - a.Cy1 : n;
    const int yp = d2 ? a.ypitch2 : a.ypitch1;
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + (lane & 15);
      uint2 v;
      v.x = pack2bf(acc[j][i][0], acc[j][i][1]);
      v.y = pack2bf(acc[j][i][2], acc[j][i][3]);
      if (m < a.M) {
        const uint32_t off = (uint32_t)(m * yp + nn) * 2u;
        if (d2) bstore8(ry2, off, v); else bstore8(ry1, off, v);
      }
      if (a.stats) {
        const float q0 = bf2f((u16)(v.x & 0xffff)), q1 = bf2f((u16)(v.x >> 16));
        const float q2 = bf2f((u16)(v.y & 0xffff)), q3 = bf2f((u16)(v.y >> 16));
        s1[j][0] += q0; s2[j][0] += q0 * q0;
        s1[j][1] += q1; s2[j][1] += q1 * q1;
        s1[j][2] += q2; s2[j][2] += q2 * q2;
        s1[j][3] += q3; s2[j][3] += q3 * q3;
      }
    }
  }
  if (a.stats) {
    // reduce over the 16 pixel lanes (lane & 15) sharing a channel group
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[j][r] += __shfl_xor(s1[j][r], o, 64);
          s2[j][r] += __shfl_xor(s2[j][r], o, 64);
        }
      }
    // combine the WAVES_M waves sharing these channels through LDS (reuse buffer 0)
    __syncthreads();
    float* red = (float*)smem;  // [WAVES_M][BN][2]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = wn * 64 + j * 16 + 4 * (lane >> 4) + r;
          red[(wm * BN + c) * 2 + 0] = s1[j][r];
          red[(wm * BN + c) * 2 + 1] = s2[j][r];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < BN; c += 256) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int q = 0; q < WAVES_M; ++q) { t1 += red[(q * BN + c) * 2]; t2 += red[(q * BN + c) * 2 + 1]; }
      a.stats[(size_t)tm * 2 * a.Cout + n0 + c] = t1;
      a.stats[(size_t)tm * 2 * a.Cout + a.Cout + n0 + c] = t2;
    }
  }
}

template <int BM, int BN>
static int launch_cfg(ConvArgs a, int variant, hipStream_t s) {
  const int tilesM = (a.M + BM - 1) / BM;
  a.tilesN = a.Cout / BN;
  if (variant == 1)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 0>), dim3(tilesM * a.tilesN), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1>), dim3(tilesM * a.tilesN), dim3(256), 0, s, a);
  return tilesM;
}

// Returns the number of M tiles (rows of the stats slab), or -1 on unsupported shape.
extern "C" int rdp_conv_igemm(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2,
                              int pitch1, int pitch2, const void* w, long wbytes, int ldw, void* y1, void* y2,
                              long ybytes1, long ybytes2, int Cy1, int ypitch1, int ypitch2, float* stats,
                              int N, int H, int W, int Cout, int taps, int packed, int bm_pref, hipStream_t s) {
  ConvArgs a;
  a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
  a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
  a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y1 = (u16*)y1; a.y2 = (u16*)y2; a.ybytes1 = (uint32_t)ybytes1; a.ybytes2 = (uint32_t)ybytes2;
  a.Cy1 = Cy1; a.ypitch1 = ypitch1; a.ypitch2 = ypitch2; a.stats = stats;
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.M = N * H * W;
  a.taps = taps; a.packed = packed;
  if (packed) {
    if (C1 != 8 || C2 != 0 || taps != 9 || ldw != 128) return -1;
    a.nks = 2; a.cpt = 1;
  } else {
    if (C1 % 64 || C2 % 64 || (taps != 9 && taps != 1)) return -1;
    a.cpt = (C1 + C2) / 64;
    a.nks = taps * a.cpt;
    if (ldw < taps * (C1 + C2)) return -1;
  }
  if (Cout % 64 || Cy1 % 4) return -1;
  if (xbytes1 >= (1l << 31) || xbytes2 >= (1l << 31) || ybytes1 >= (1l << 31) || ybytes2 >= (1l << 31)) return -1;
  // bm_pref: 0 = auto, 128 / 256 = force tile; +1000 * variant selects the LDS layout (A/B tests)
  const int variant = bm_pref / 1000;
  bm_pref %= 1000;
  if ((bm_pref == 128 || bm_pref == 0) && Cout % 128 == 0) return launch_cfg<128, 128>(a, variant, s);
  return launch_cfg<256, 64>(a, variant, s);
}
