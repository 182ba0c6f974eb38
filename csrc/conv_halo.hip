// 3x3 convolution (stride 1, pad 1), NHWC bf16, as a halo-tiled direct convolution on MFMA.
//
// Same contract as conv_igemm.hip (forward and dgrad of /root/reference/pkg/segmentation_model.py
// DoubleConv convs, two concatenated input sources, split output, fused BN-stats / BN-fold
// epilogue), different data movement:
//
//   implicit GEMM (conv_igemm.hip): every K step (tap, 64 channels) re-fetches the tile's 128-256
//     pixel rows shifted by the tap, so each activation line crosses L2->LDS 9 times; at ~256 B of
//     LDS-DMA per MFMA that kernel runs at the L2->LDS gather rate (~17-19 TB/s chip-wide,
//     MI355X_MICROARCH.md "Indexed rows"), not at the MFMA rate.
//   halo tile (this file): a block owns TR x TC output pixels (256) x BN output channels. For each
//     64-channel input chunk the (TR+2) x (TC+2) halo tile is staged ONCE into LDS; the 9 taps read
//     it at shifted row offsets. Only the weight slice (BN x 64 ch of one tap) streams per K step.
//     L2->LDS bytes per MFMA drop ~3x (BN=128: 16 KB weights + ~5.6 KB halo per 256 MFMAs).
//
// LDS images are row-major [row][128 B] with the 16-B chunk XOR-swizzled by (row & 7) on the
// SOURCE address (LDS-DMA writes lane-linear). Halo rows are consecutive pixels of the padded tile,
// so a tap shift is a uniform row offset and fragment reads of 16 consecutive pixels stay
// bank-conflict free (the swizzle is a rotation over any 8 consecutive rows).
//
// Measured (scripts/conv_microbench.py, bs32 U-Net shapes): despite ~3x fewer L2->LDS bytes this
// kernel beats conv_igemm only for 64-channel outputs with >= 256 input channels (556 vs 469 TF/s
// at 128x128, 256->64); elsewhere it is 10-30 % slower. PMC shows both kernels at ~40 % MFMA-busy:
// the limiter is per-step latency (barrier + DMA + LDS read before the first MFMA), which
// conv_igemm hides with two independent 4-wave blocks per CU, while this kernel needs > 80 KB of
// LDS and runs one 8-wave block per CU whose waves hit each barrier in lockstep. The dispatcher in
// conv_igemm.hip selects it only where it measured faster.
//
// Pipeline: one continuous step sequence over (tile, chunk, tap); one s_barrier per step. At step
// s the block issues the weight slice of step s+2 (3-slot ring, counted vmcnt) and 1/8 of the NEXT
// chunk's halo tile (spread over taps 0..7 so the L2->LDS rate stays flat).
#include "common.h"

struct HaloArgs {
  const u16* x1;
  const u16* x2;
  uint32_t xbytes1, xbytes2;
  int C1, C2, pitch1, pitch2;
  const u16* w;
  uint32_t wbytes;
  int ldw, cin;  // weight row length; total input channels (tap stride in a weight row)
  u16* y1;
  u16* y2;
  uint32_t ybytes1, ybytes2;
  int Cy1, ypitch1, ypitch2;
  float* stats;
  const float* escale;
  const float* eshift;
  int erelu;
  int N, H, W, Cout;
  int nchunks;           // input 64-channel chunks
  int tilesH, tilesW, tilesN, ntiles;
};

template <int TC, int TR, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_halo_kernel(const HaloArgs a) {
  constexpr int NW = WM * WN;
  constexpr int RUN = (TC * TR) / WM;  // pixels per wave (consecutive in tile row-major order)
  constexpr int NI = RUN / 16;         // 16-pixel fragments per wave
  constexpr int HC = TC + 2, HR = TR + 2, HROWS = HC * HR;
  constexpr int P = (HROWS + 7) / 8;             // 1-KiB DMA pieces per halo tile
  constexpr int PPT = (P + 8 * NW - 1) / (8 * NW);  // halo pieces per wave per step (taps 0..7)
  constexpr int A_BYTES = P * 1024;
  constexpr int BN = 64 * WN;
  constexpr int W_BYTES = BN * 128;
  constexpr int WPW = BN / 8 / NW;  // weight pieces per wave per step
  constexpr int WSLOTS = 3;  // weight ring: slice s+2 is issued while slice s is consumed
  constexpr int JUNK = 1024;  // LDS sink for the fixed-count halo issue (pieces past the tile)
  static_assert(TC % 16 == 0 && RUN % 16 == 0 && WPW >= 1, "tile shape");
  static_assert(2 * A_BYTES + WSLOTS * W_BYTES + JUNK <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + WSLOTS * W_BYTES + JUNK];
  char* const abuf0 = smem;
  char* const wbuf0 = smem + 2 * A_BYTES;
  char* const junk = smem + 2 * A_BYTES + WSLOTS * W_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int gch = (lane & 7) ^ (lane >> 3);  // 16-B chunk fetched by this lane (row & 7 == lane >> 3)

  const uint32_t G = gridDim.x;
  const uint32_t lid = xcd_remap(blockIdx.x, G);
  const int my_tiles = lid < (uint32_t)a.ntiles ? (a.ntiles - 1 - (int)lid) / (int)G + 1 : 0;
  const int steps_per_tile = a.nchunks * 9;
  const int total = my_tiles * steps_per_tile;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);

  // ---- halo (A) stream state: pixel index (or -1) of every piece row this wave loads ----
  int apix[8 * PPT];
  auto set_atile = [&](int t) {
    const int tile = (int)lid + t * (int)G;
    const int tm = tile / a.tilesN;
    const int tw = tm % a.tilesW, t2 = tm / a.tilesW;
    const int th = t2 % a.tilesH, n = t2 / a.tilesH;
    const int h0 = th * TR - 1, w0 = tw * TC - 1;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int p = (s * NW + wave) * PPT + k;
        const int hp = p * 8 + (lane >> 3);
        const int hr = hp / HC, hc = hp - (hp / HC) * HC;
        const int h = h0 + hr, w = w0 + hc;
        const bool ok = (p < P) & (hp < HROWS) & inb(h, a.H) & inb(w, a.W);
        apix[s * PPT + k] = ok ? (n * a.H + h) * a.W + w : -1;
      }
  };
  // Every wave issues exactly PPT pieces per call (pieces past the tile go to the junk slot), so
  // the number of vector-memory ops per step is a compile-time constant for the counted vmcnt.
  auto issue_a = [&](int part, int chunk, char* buf) {
    const int c0 = chunk * 64;
    const bool s2 = c0 >= a.C1;
    const int pitch = s2 ? a.pitch2 : a.pitch1;
    const int coff = (s2 ? c0 - a.C1 : c0) + gch * 8;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s != part) continue;  // part is wave-uniform: selects one register group without indexing
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int p = (s * NW + wave) * PPT + k;
        const int px = apix[s * PPT + k];
        const uint32_t off = px >= 0 ? (uint32_t)(px * pitch + coff) * 2u : RDP_OOB;
        dma16(s2 ? rx2 : rx1, (lds_void*)(p < P ? buf + p * 1024 : junk), off);
      }
    }
  };
  auto issue_a_none = [&]() {
#pragma unroll
    for (int k = 0; k < PPT; ++k) dma16(rx1, (lds_void*)junk, RDP_OOB);
  };
  // ---- weight stream: rows n = tn*BN + (wave*WPW + f)*8 + (lane>>3) ----
  auto issue_w = [&](int tn, int chunk, int tap, char* buf) {
    const uint32_t kofs = (uint32_t)(tap * a.cin + chunk * 64 + gch * 8);
#pragma unroll
    for (int f = 0; f < WPW; ++f) {
      const int n = tn * BN + (wave * WPW + f) * 8 + (lane >> 3);
      dma16(rw, (lds_void*)(buf + (wave * WPW + f) * 1024), ((uint32_t)n * (uint32_t)a.ldw + kofs) * 2u);
    }
  };

  // ---- fragment read geometry ----
  const int l16 = lane & 15, kq = lane >> 4;
  int hpb[NI];  // halo row of this lane's pixel for tap (1,1) (centre), fragment i
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int t0 = wm * RUN + 16 * i;
    const int r = t0 / TC, c = t0 % TC;
    hpb[i] = (r + 1) * HC + (c + 1) + l16;
  }
  int wro[4];  // weight fragment LDS offsets (k-half 0)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wn * 64 + 16 * j + l16;
    wro[j] = row * 128 + 16 * (kq ^ (row & 7));
  }

  const auto ry1 = make_rsrc(a.y1, a.ybytes1);
  const auto ry2 = make_rsrc(a.y2 ? a.y2 : a.y1, a.y2 ? a.ybytes2 : 0u);

  f32x4 acc[4][NI];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // cursors: A stream loads chunk q+1 while chunk q computes; W stream runs one step ahead
  int a_t = 0, a_c = 0;           // tile (local index) / chunk of the halo being loaded
  int w_t = 0, w_c = 0, w_tap = 0;  // step being loaded for the weights
  auto tn_of = [&](int t) { return ((int)lid + t * (int)G) % a.tilesN; };

  if (total > 0) {
    set_atile(0);
#pragma unroll
    for (int s = 0; s < 8; ++s) issue_a(s, 0, abuf0);
    // the A cursor now points at the chunk after (tile 0, chunk 0)
    if (++a_c == a.nchunks) { a_c = 0; ++a_t; if (a_t < my_tiles) set_atile(a_t); }
    issue_w(tn_of(0), 0, 0, wbuf0);
    // W cursor -> step 1
    if (++w_tap == 9) { w_tap = 0; if (++w_c == a.nchunks) { w_c = 0; ++w_t; } }
    issue_w(total > 1 ? tn_of(w_t) : 0, w_c, w_tap, wbuf0 + W_BYTES);  // (dummy if total == 1)
    issue_a_none();
  }
  int t = 0, c = 0, tap = 0;  // compute cursor
  int q = 0;                  // flattened chunk index of the compute cursor
  constexpr int PER_STEP = WPW + PPT;  // vector-memory ops each wave issues per step
  for (int s = 0; s < total; ++s) {
    // step s needs W(s) (issued two steps ago) and its halo chunk (issued during the previous
    // chunk, at taps 0..7): everything but the youngest step's issues must have landed
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STEP) : "memory");
    raw_barrier();
    // ---- issue: weights of step s+2, part `tap` of the next chunk's halo (taps 0..7) ----
    if (s + 2 < total) {
      if (++w_tap == 9) { w_tap = 0; if (++w_c == a.nchunks) { w_c = 0; ++w_t; } }
      issue_w(tn_of(w_t), w_c, w_tap, wbuf0 + ((s + 2) % WSLOTS) * W_BYTES);
    } else {
      issue_w(0, 0, 0, wbuf0 + ((s + 2) % WSLOTS) * W_BYTES);  // dummy (slot never read again)
    }
    if (tap < 8 && a_t < my_tiles) issue_a(tap, a_c, abuf0 + ((q + 1) & 1) * A_BYTES);
    else issue_a_none();

    // ---- compute step s ----
    const char* ab = abuf0 + (q & 1) * A_BYTES;
    const char* wb = wbuf0 + (s % WSLOTS) * W_BYTES;
    const int shift = ((tap * 11 >> 5) - 1) * HC + (tap - 3 * (tap * 11 >> 5)) - 1;
    int ao[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int hp = hpb[i] + shift;
      ao[i] = hp * 128 + 16 * (kq ^ (hp & 7));
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bf16x8 fa[4], fb[NI];
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[j] = *(const bf16x8*)(wb + (wro[j] ^ (hf * 64)));
#pragma unroll
      for (int i = 0; i < NI; ++i) fb[i] = *(const bf16x8*)(ab + (ao[i] ^ (hf * 64)));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
    }
    // advance the compute cursor (and the A cursor at chunk boundaries)
    if (++tap < 9) continue;
    tap = 0;
    ++q;
    if (a_t < my_tiles) {
      if (++a_c == a.nchunks) { a_c = 0; ++a_t; if (a_t < my_tiles) set_atile(a_t); }
    }
    if (++c < a.nchunks) continue;
    c = 0;

    // ---- epilogue of tile t ----
    const int tile = (int)lid + t * (int)G;
    ++t;
    const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
    const int tw = tm % a.tilesW, t2 = tm / a.tilesW;
    const int th = t2 % a.tilesH, n = t2 / a.tilesH;
    const int n0 = tn * BN;
    float s1[4][4], s2[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nc = n0 + wn * 64 + j * 16 + 4 * kq;
      const bool d2 = nc >= a.Cy1;
      const int nn = d2 ? nc - a.Cy1 : nc;
      const int yp = d2 ? a.ypitch2 : a.ypitch1;
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
      float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a.escale) { sc = *(const float4*)(a.escale + nc); sh = *(const float4*)(a.eshift + nc); }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int tp = wm * RUN + 16 * i + l16;
        const int r = tp / TC, cc = tp % TC;
        const int m = (n * a.H + th * TR + r) * a.W + tw * TC + cc;
        f32x4 o = acc[j][i];
        if (a.escale) {
          o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
          o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
          if (a.erelu) {
            o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
          }
        }
        uint2 v;
        v.x = pack2bf(o[0], o[1]);
        v.y = pack2bf(o[2], o[3]);
        acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        bstore8(d2 ? ry2 : ry1, (uint32_t)(m * yp + nn) * 2u, v);
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
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] = row16_sum(s1[j][r]);
          s2[j][r] = row16_sum(s2[j][r]);
        }
      if (l16 == 0) {
        float* row = a.stats + (size_t)(tm * WM + wm) * 2 * a.Cout;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cc = n0 + wn * 64 + j * 16 + 4 * kq;
          *(float4*)(row + cc) = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
          *(float4*)(row + a.Cout + cc) = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
        }
      }
    }
  }
  // no LDS-DMA (dummy weight / halo sink loads) may still be in flight when LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int TC, int TR, int WM, int WN>
static int halo_launch(HaloArgs a, hipStream_t s) {
  a.tilesH = a.H / TR;
  a.tilesW = a.W / TC;
  a.tilesN = a.Cout / (64 * WN);
  const int tilesM = a.N * a.tilesH * a.tilesW;
  a.ntiles = tilesM * a.tilesN;
  const int grid = a.ntiles < 256 ? a.ntiles : 256;
  hipLaunchKernelGGL((conv_halo_kernel<TC, TR, WM, WN>), dim3(grid), dim3(64 * WM * WN), 0, s, a);
  return tilesM * WM;
}

// Number of 256-pixel output tiles x cout tiles the halo kernel would use (0 = shape unsupported).
extern "C" int rdp_conv_halo_tiles(int N, int H, int W, int C1, int C2, int Cout, int taps, int packed) {
  if (taps != 9 || packed || C1 % 64 || C2 % 64 || C1 == 0 || Cout % 64) return 0;
  int tc, tr;
  if (W % 64 == 0 && H % 4 == 0) { tc = 64; tr = 4; }
  else if (W % 32 == 0 && H % 8 == 0) { tc = 32; tr = 8; }
  else if (W % 16 == 0 && H % 16 == 0) { tc = 16; tr = 16; }
  else return 0;
  const int wn = Cout % 128 == 0 ? 2 : 1;
  return N * (H / tr) * (W / tc) * (Cout / (64 * wn));
}

// Returns stats rows written (>= 0) or -1 if unsupported.
extern "C" int rdp_conv_halo(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2, int pitch1,
                             int pitch2, const void* w, long wbytes, int ldw, void* y1, void* y2, long ybytes1,
                             long ybytes2, int Cy1, int ypitch1, int ypitch2, float* stats, int N, int H, int W,
                             int Cout, const float* escale, const float* eshift, int erelu, hipStream_t s) {
  if (!rdp_conv_halo_tiles(N, H, W, C1, C2, Cout, 9, 0)) return -1;
  if (ldw < 9 * (C1 + C2) || Cy1 % 4) return -1;
  if (xbytes1 >= (1l << 31) || xbytes2 >= (1l << 31) || ybytes1 >= (1l << 31) || ybytes2 >= (1l << 31) ||
      wbytes >= (1l << 31))
    return -1;
  HaloArgs a;
  a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
  a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
  a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw; a.cin = C1 + C2;
  a.y1 = (u16*)y1; a.y2 = (u16*)y2; a.ybytes1 = (uint32_t)ybytes1; a.ybytes2 = (uint32_t)ybytes2;
  a.Cy1 = Cy1; a.ypitch1 = ypitch1; a.ypitch2 = ypitch2;
  a.stats = stats; a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  a.N = N; a.H = H; a.W = W; a.Cout = Cout;
  a.nchunks = (C1 + C2) / 64;
  const bool wide = Cout % 128 == 0;
  // 8 waves per block either way (2 per SIMD): BN=128 -> 4 (pixels) x 2 (couts), BN=64 -> 8 x 1
  if (W % 64 == 0 && H % 4 == 0) return wide ? halo_launch<64, 4, 4, 2>(a, s) : halo_launch<64, 4, 8, 1>(a, s);
  if (W % 32 == 0 && H % 8 == 0) return wide ? halo_launch<32, 8, 4, 2>(a, s) : halo_launch<32, 8, 8, 1>(a, s);
  return wide ? halo_launch<16, 16, 4, 2>(a, s) : halo_launch<16, 16, 8, 1>(a, s);
}
