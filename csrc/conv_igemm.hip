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
//     training-mode BatchNorm: one slab row per (M tile, wave row), reduced by bn_finalize.
//
// Tiling: block = 4 waves (256 threads), block tile BM x BN with each wave owning 64x64; K step
// = 64 channels of one tap. Both operand tiles are staged global->LDS by LDS-DMA
// (buffer_load ... lds, 16 B/lane) as a row-major [rows][128 B] image: one wave-instruction moves
// 8 full 128-B lines, with the 16-B chunk XOR-swizzled by (row & 7) on the SOURCE address so the
// MFMA-fragment ds_read_b128s are bank-conflict free. (A fragment-shaped image -- 16 rows x 64 B
// per instruction -- doubles the TA line lookups and ran 1.4-1.6x slower on deep layers.)
// Halo/zero padding comes from out-of-range buffer offsets (hardware returns 0).
//
// Persistent: each block walks several output tiles with ONE continuous double-buffered K
// pipeline (one raw s_barrier per K step), so tile t+1's first DMA lands under tile t's last
// MFMAs and epilogue. This removes the per-tile prologue that dominated the small-K (K = 576)
// 64-channel layers. The epilogue uses no LDS and no block barrier.
#include "common.h"
#include <stdlib.h>

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
  float* stats;  // [tilesM * WAVES_M][2][Cout] partial (sum, sumsq) or nullptr
  const float* escale;  // eval-mode BN fold: out = relu?(acc * escale[n] + eshift[n]) (or nullptr)
  const float* eshift;
  int erelu;
  int N, H, W, Cout, M;
  int taps;  // 9 (3x3) or 1 (1x1)
  int packed;  // 1: Cin == 8, K packs 8 taps per 64-wide K step
  int nks;  // number of K steps per work item (= per tile unless split-K)
  int cpt;  // 64-channel chunks per tap (generic mode)
  int ksplit;    // > 1: split-K, work item = (tile, split), fp32 partial tiles go to kslab
  float* kslab;  // [ksplit][M][Cout] fp32
  u16* pool;       // split-K reduce only: also write MaxPool2d(2) of the output (eval), [M/4][ppitch]
  int ppitch;
  // split-K reduce only: also write the bilinear x2 (align_corners) upsample of the output (eval), into
  // up [N][uH][uW][upitch] at offset (uoy, uox) (F.pad of the decoder), zeros outside
  u16* up;
  int upitch, uH, uW, uoy, uox;
  float urh, urw;
  int tilesN, ntiles;
  uint32_t fhw_m, fhw_s, fw_m, fw_s;  // magic division by H*W and by W
  // ConvTranspose2d(k=2, s=2) output written in place (ping-pong epilogue, rdp_conv_upT_fwd): GEMM
  // column n = sub * 2^tlc + c of low-res pixel (img, h, w) goes to y1 pixel (img, 2h + sub/2 + toy,
  // 2w + sub%2 + tox) of a [N][tH2][tW2] map, channel c, + ubias[c]. tlc = 0: plain output.
  const float* ubias = nullptr;
  int tlc = 0, tH2 = 0, tW2 = 0, toy = 0, tox = 0;
  // split-K reduce only (training dgrad, one destination): the BN-backward partial rows of the BN + ReLU
  // layer whose activation gradient this conv writes, in bn_relu_bwd_reduce's layout -- bnpart[block][0][c]
  // = sum g, [block][1][c] = sum g * xhat, g = out * (bny * scale + shift > 0), xhat = (bny - mean) * invstd
  // -- so the standalone reduce pass (reading the output and bny back) disappears
  const u16* bny = nullptr;       // that layer's pre-BN output
  const float* bncoef = nullptr;  // its [mean | invstd | scale | shift]
  float* bnpart = nullptr;
  int bnypitch = 0;
  int* bnrows = nullptr;  // host cell: the partial rows written (set when the split-K reduce ran)
};

// 128 -> 128 convs as two two-source-ring launches where the ring grid is at least this large. Measured
// (scripts/conv_microbench.py --shapes 2, one MI355X): 128^2 128 -> 128 at bs 64 330.5 vs 368.9 us for the
// 256 x 128 ping-pong kernel, but 106.8 vs 98.5 at bs 16 and 45.8 vs 28.3 at bs 4 (each launch reads the
// whole input); bs-64 step 19.43 / 19.55 vs 19.47 / 19.61 ms (interleaved).
constexpr long RING2_X2_PAIRS = 4096;

// tap (0..8) -> (dr, ds) without division: dr + 1 = (tap * 11) >> 5
RDP_DEV int tap_dr(int tap) { return ((tap * 11) >> 5) - 1; }
RDP_DEV int tap_ds(int tap) { return tap - 3 * ((tap * 11) >> 5) - 1; }

template <int N>
RDP_DEV void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
// wait until at most B + (epilogue stores issued since) vector-memory ops are outstanding
template <int B, int P1, int P2>
RDP_DEV void vm_wait_p(int pend) {
  if (pend == 0) vm_wait<B>();
  else if (pend == P1) vm_wait<B + P1>();
  else vm_wait<B + P2>();
}

// Double-buffered K pipeline at 2 blocks / CU: the co-resident block hides the DMA latency. (A 3-4
// stage ring at 1 block / CU and an in-kernel split-K fixup were measured slower: profiles/dead_ends.md.)
template <int BM, int BN, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 2) void conv_igemm_kernel(const ConvArgs a) {
  constexpr int NST = 2;
  constexpr int WAVES_M = BM / 64;
  constexpr int WAVES_N = NWV / WAVES_M;
  constexpr int WNT = BN / WAVES_N;  // couts per wave (64, or 32 with 8-wave blocks)
  constexpr int NJ = WNT / 16;
  constexpr int P_BYTES = BM * 128, W_BYTES = BN * 128, BUF = P_BYTES + W_BYTES;
  constexpr int NROW = BM / 8 / NWV;     // pixel-row DMA pieces per wave per K step
  constexpr int WPIECES = BN / 8 / NWV;  // weight-row DMA pieces per wave per K step
  constexpr int DMA_OPS = NROW + WPIECES;  // vector-memory ops per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NST * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int gch = (lane & 7) ^ (lane >> 3);  // global 16-B chunk this lane fetches (row-major image)

  const uint32_t G = gridDim.x;
  const uint32_t lid = xcd_remap(blockIdx.x, G);
  const int my_tiles = lid < (uint32_t)a.ntiles ? (a.ntiles - 1 - (int)lid) / (int)G + 1 : 0;
  const int total = my_tiles * a.nks;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);

  // ---- DMA-side state of the tile currently being staged ----
  // per pixel row (computed once per tile): byte offset of this lane's 16-B chunk of the pixel in
  // each source (pb1 / pb2), and the INVERTED 9-bit tap mask (bit t set <=> row invalid or
  // (h+dr, w+ds) outside the image). The per-K-step address is then 3 full-rate VALU ops per DMA:
  // v_bfe (tap bit) + v_add (uniform tap/channel offset) + v_lshl_or (bit 31 = out of range, which
  // the buffer descriptor turns into zeros) -- no multiply or compare in the K loop.
  uint32_t pb1[NROW], pb2[NROW];
  uint32_t nmask[NROW];
  uint32_t woff[WPIECES];
  int itap = 0, icc = 0;  // (tap, 64-channel chunk) of the stage being issued (generic mode)
  int ks0 = 0;  // first global K step of the work item being staged (split-K)
  auto set_tile = [&](int t) {
    const int item = (int)lid + t * (int)G;
    const int tile = a.ksplit > 1 ? item % (a.ntiles / a.ksplit) : item;
    ks0 = a.ksplit > 1 ? (item / (a.ntiles / a.ksplit)) * a.nks : 0;
    itap = ks0 / a.cpt;
    icc = ks0 - itap * a.cpt;
    const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      const int m = tm * BM + (wave * NROW + r) * 8 + (lane >> 3);
      const bool valid = m < a.M;
      const uint32_t mm = valid ? (uint32_t)m : 0u;
      const uint32_t hw = mm - ((__umulhi(mm, a.fhw_m) + mm) >> a.fhw_s) * (uint32_t)(a.H * a.W);
      const uint32_t h = (__umulhi(hw, a.fw_m) + hw) >> a.fw_s;
      const uint32_t w = hw - h * (uint32_t)a.W;
      // rows allowed: dr=-1 needs h>0, dr=+1 needs h<H-1; same for columns
      const uint32_t rok = (h > 0 ? 1u : 0u) | 2u | (h + 1 < (uint32_t)a.H ? 4u : 0u);
      const uint32_t cok = (w > 0 ? 1u : 0u) | 2u | (w + 1 < (uint32_t)a.W ? 4u : 0u);
      // tap = 3*(dr+1) + (ds+1): mask = rows (x) cols outer product
      uint32_t msk = 0;
      msk |= (rok & 1u) ? cok : 0u;
      msk |= (rok & 2u) ? (cok << 3) : 0u;
      msk |= (rok & 4u) ? (cok << 6) : 0u;
      if (a.taps == 1) msk = 1u;
      nmask[r] = valid ? ~msk : ~0u;
      pb1[r] = (mm * (uint32_t)a.pitch1 + (uint32_t)gch * 8u) * 2u;
      pb2[r] = (mm * (uint32_t)a.pitch2 + (uint32_t)gch * 8u) * 2u;
    }
#pragma unroll
    for (int f = 0; f < WPIECES; ++f) {
      const int n = tn * BN + (wave * WPIECES + f) * 8 + (lane >> 3);
      woff[f] = (uint32_t)(n * a.ldw + gch * 8) * 2u;
    }
  };

  auto issue = [&](int ks, char* buf) {
    if (a.packed) {
      const int tap = ks * 8 + gch;  // per lane; taps >= 9 have no mask bit -> zeros
      const int toff = (tap_dr(tap) * a.W + tap_ds(tap)) * a.pitch1 * 2 - gch * 16;
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        const uint32_t bad = tap < 9 ? (nmask[r] >> tap) & 1u : 1u;
        const uint32_t off = (bad << 31) | (uint32_t)((int)pb1[r] + toff);
        dma16(rx1, (lds_void*)(buf + (wave * NROW + r) * 1024), off);
      }
    } else {
      const int c0 = icc * 64;
      const bool s2 = c0 >= a.C1;
      const int pitch = s2 ? a.pitch2 : a.pitch1;
      const int tap_lin = a.taps == 9 ? tap_dr(itap) * a.W + tap_ds(itap) : 0;
      const int soff = (tap_lin * pitch + (s2 ? c0 - a.C1 : c0)) * 2;  // wave-uniform (SGPR)
      const int bit = a.taps == 9 ? itap : 0;
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        const uint32_t bad = __builtin_amdgcn_ubfe(nmask[r], (uint32_t)bit, 1u);
        const uint32_t off = (bad << 31) | (uint32_t)((int)(s2 ? pb2[r] : pb1[r]) + soff);
        dma16(s2 ? rx2 : rx1, (lds_void*)(buf + (wave * NROW + r) * 1024), off);
      }
      if (++icc == a.cpt) { icc = 0; ++itap; if (itap == a.taps) itap = 0; }
    }
    char* wbuf = buf + P_BYTES;
#pragma unroll
    for (int f = 0; f < WPIECES; ++f)
      dma16(rw, (lds_void*)(wbuf + (wave * WPIECES + f) * 1024), woff[f] + (uint32_t)(ks0 + ks) * 128u);
  };

  // LDS byte offsets of this lane's fragment reads (k-half hf) relative to a 16-row subtile
  int rdoff[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) rdoff[hf] = (lane & 15) * 128 + 16 * (((lane >> 4) + 4 * hf) ^ (lane & 7));

  const auto ry1 = make_rsrc(a.y1, a.ybytes1);
  const auto ry2 = make_rsrc(a.y2 ? a.y2 : a.y1, a.y2 ? a.ybytes2 : 0u);

  f32x4 acc[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  int ks = 0, t = 0;    // compute position (K step within tile, tile index)
  int iks = 0, it = 0;  // issue position (K step within tile, tile index) of the newest stage
  int ig = 0;           // global index of the newest issued stage
  int ibuf = 0, cbuf = 0;  // LDS buffer of the newest issued stage / of the stage being computed
  if (total > 0) {
    set_tile(0);
    issue(0, smem);
  }
  // vector-memory stores the previous step's epilogue issued after stage g's DMA: vmcnt counts
  // them in issue order, so stage g has landed once at most that many ops are outstanding (a plain
  // vmcnt(0) would also wait for the output stores of every tile before its next K step)
  int pend = 0;
  // Training BN statistics accumulate over ALL of this block's tiles: with the persistent grid a
  // multiple of tilesN (host-checked), block lid always has channel tile tn = lid % tilesN, so one
  // slab row per (lid / tilesN, wm) -- grid * WAVES_M / tilesN rows instead of one per M-tile
  // (65536 at 256^2 x 64 ch, bs 64), written once after the last tile.
  float s1[NJ][4], s2[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
  for (int g = 0; g < total; ++g) {
    // stage g has landed once at most (epilogue stores issued after it) ops are outstanding
    // (in-order completion); older stores are not counted, which only makes the wait stricter
    vm_wait_p<0, 2 * NJ, 4 * NJ>(pend);
    pend = 0;
    raw_barrier();
    if (ig + 1 < total) {  // the buffer computed at step g-1: every wave is past it (barrier above)
      if (++iks == a.nks) { iks = 0; ++it; set_tile(it); }
      ibuf = ibuf + 1 == NST ? 0 : ibuf + 1;
      issue(iks, smem + ibuf * BUF);
      ++ig;
    }
    const char* pb = smem + cbuf * BUF;
    cbuf = cbuf + 1 == NST ? 0 : cbuf + 1;
    const char* wb = pb + P_BYTES;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bf16x8 fa[NJ], fb[4];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fa[j] = *(const bf16x8*)(wb + (wn * NJ + j) * 2048 + rdoff[hf]);
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = *(const bf16x8*)(pb + (wm * 4 + i) * 2048 + rdoff[hf]);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[j], fb[i], acc[j][i], 0, 0, 0);
    }
    if (++ks < a.nks) continue;

    // ---- epilogue of tile t: acc[j][i][r] = out[m = m0 + wm*64 + 16i + (lane&15)][n = n0 + wn*64 + 16j + 4*(lane>>4) + r]
    ks = 0;
    const int item = (int)lid + t * (int)G;
    ++t;
    int tile = item;
    if (a.ksplit > 1) {  // fp32 partial tile -> slab[split][m][n]
      const int tiles1 = a.ntiles / a.ksplit;
      tile = item % tiles1;
      const int split = item / tiles1;
      const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
      const auto rk = make_rsrc(a.kslab, (uint32_t)((long)a.ksplit * a.M * a.Cout * 4));
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = tn * BN + wn * WNT + j * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = tm * BM + wm * 64 + i * 16 + (lane & 15);
          const f32x4 o = acc[j][i];
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          const uint32_t off = m < a.M ? (uint32_t)(((long)split * a.M + m) * a.Cout + n) * 4u : RDP_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rk, off, 0, 0);
        }
      }
      pend = 4 * NJ;  // NJ x 4 slab stores; the epilogue runs in conv_splitk_reduce_kernel
      continue;
    }
    const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
    const int m0 = tm * BM, n0 = tn * BN;
    // Widened stores: a lane holds 4 couts (16 j + 4 g + r, g = lane >> 4) of one pixel per
    // fragment. v_permlane16_swap of fragment pair (j, j+1) gives every lane 8 consecutive couts
    // (lanes g: 0 -> 0..7, 1 -> 16..23, 2 -> 8..15, 3 -> 24..31 of the pair) = one 16-B store, and a
    // pixel's 32 couts become 64 contiguous bytes per instruction (cdna_hip_programming.md T21).
    const int gq = lane >> 4;
    const int coff = 16 * (gq & 1) + 8 * (gq >> 1);
#pragma unroll
    for (int jp = 0; jp < NJ; jp += 2) {
      const int nb = n0 + wn * WNT + jp * 16;  // first cout of the pair
      const int n = nb + coff;                  // this lane's 8 couts after the swap
      const bool d2 = n >= a.Cy1;
      const int nn = d2 ? n - a.Cy1 : n;
      const int yp = d2 ? a.ypitch2 : a.ypitch1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + (lane & 15);
        uint2 v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = jp + h;
          f32x4 o = acc[j][i];
          if (a.escale) {
            const int nc = nb + h * 16 + 4 * gq;
            const float4 sc = *(const float4*)(a.escale + nc), sh = *(const float4*)(a.eshift + nc);
            o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
            o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
            if (a.erelu) {
              o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
            }
          }
          v[h].x = pack2bf(o[0], o[1]);
          v[h].y = pack2bf(o[2], o[3]);
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (a.stats) {
            const float q0 = __uint_as_float(v[h].x << 16), q1 = __uint_as_float(v[h].x & 0xffff0000u);
            const float q2 = __uint_as_float(v[h].y << 16), q3 = __uint_as_float(v[h].y & 0xffff0000u);
            s1[j][0] += q0; s2[j][0] += q0 * q0;
            s1[j][1] += q1; s2[j][1] += q1 * q1;
            s1[j][2] += q2; s2[j][2] += q2 * q2;
            s1[j][3] += q3; s2[j][3] += q3 * q3;
          }
        }
        const auto rxs = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
        const auto rys = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
        const uint32_t off = m < a.M ? (uint32_t)(m * yp + nn) * 2u : RDP_OOB;
        bstore16(d2 ? ry2 : ry1, off, make_uint4(rxs[0], rys[0], rxs[1], rys[1]));
      }
    }
    pend = 2 * NJ;  // 2 NJ output stores
  }
  if (a.stats && a.ksplit == 1 && total > 0) {
    // reduce over the 16 pixel lanes (lane & 15) sharing a channel group; one slab row per (block group, wm)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] = row16_sum(s1[j][r]);
        s2[j][r] = row16_sum(s2[j][r]);
      }
    if ((lane & 15) == 0) {
      const int tn = (int)lid % a.tilesN;
      float* row = a.stats + (size_t)(((int)lid / a.tilesN) * WAVES_M + wm) * 2 * a.Cout;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = tn * BN + wn * WNT + j * 16 + 4 * (lane >> 4);
        *(float4*)(row + c) = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
        *(float4*)(row + a.Cout + c) = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong 256 x BN tile (BN = 256 or 128): 8 waves, ONE block per CU, 2-3 stage K ring.
//
// The 2-barrier structure above (2 blocks / CU, 128 x 128 tiles) tops out near 0.9-1.1 PF: every
// K step waits for its own stage behind one barrier, with about one K step of MFMA work to hide
// the DMA. Here the two wave groups of the block (wm = 0: waves 0-3, wm = 1: waves 4-7; one wave
// of each group per SIMD) run staggered by one barrier (cdna_hip_programming.md "The 256^2 8-phase
// template", T3+T4+T5): while one group issues its LDS fragment reads and DMA, its partner on the
// same SIMD runs a 16-MFMA cluster. A K step (64 channels of one tap) is NPH phases; a phase is a
// memory segment (fragment reads [+ the DMA of a later stage at phase 0] + lgkmcnt(0)) and a
// compute segment (16 MFMAs), each ended by one raw s_barrier. Stage g+NST-1 is issued at phase 0
// of K step g and waited for (counted vmcnt, never a drain of newer stages) in the memory segment
// of the last phase of K step NST-2 later, i.e. 1.5 K steps (NST 2) to 2.5 K steps (NST 3) of
// MFMA work hide each DMA -- and the 256-wide tile halves the LDS fill bytes per FLOP of the
// 128 x 128 tile. Ordering (one barrier more than unstaggered, as the template requires):
//   * RAW: each wave waits for its own DMA of stage g+1 in M(g, NPH-1); group 1 runs that segment
//     one slot later than group 0, i.e. in the slot just before group 0's first read M(g+1, 0).
//   * WAR: every memory segment ends with lgkmcnt(0), so the last reads of a buffer (M(g-1,
//     NPH-1), group 1 one slot later) are complete before the barrier that precedes the first DMA
//     into it (M(g, 0) of group 0).
// Accumulation order per output element is the K-step order with the two K halves of a step in
// order, exactly as conv_igemm_kernel: outputs are bitwise equal to it. Training BN statistics
// accumulate per block in LDS words owned by one lane each (no registers held across tiles).
// Generic (non-packed) im2col only, no split-K / fused pool or upsample.
// Fragment reads of phases 0..NPH-2 stay in flight across the segment barrier; at BN = 256 both
// cout halves of the weight fragments stay in registers (HOLDB: no re-read in phase 3); BN = 128
// runs a 3-stage K ring (NST). (A 512 x 64 form and a BN-backward reduction in the dgrad epilogue
// were measured slower: profiles/dead_ends.md.)
// UT: ConvTranspose2d sub-pixel output (ConvArgs tlc / ubias; no stats, no split); UTR: the
// ConvTranspose2d input gradient, the A operand read at the 4 sub-pixels of the output gradient
// (taps = 4, ConvArgs tH2 / tW2 / toy / tox) -- their own instantiations, so the plain kernels'
// scalar registers are untouched.
template <int BN, bool SPLIT = false, bool UT = false, bool UTR = false>
__global__ __launch_bounds__(512, 1) void conv_pp_kernel(const ConvArgs a) {
  // 256-pixel tile, wave (wm, wn) = 128 pixels x BN/4 couts
  constexpr int NST = BN == 128 ? 3 : 2;
  constexpr bool RD_INFLIGHT = true, HOLDB = BN == 256;
  constexpr int BM = 256;
  constexpr int WNT = BN / 4;        // couts per wave
  constexpr int NJ = WNT / 16;       // cout fragments per wave (4 / 2)
  constexpr int NI = 8;              // pixel fragments per wave
  constexpr int NPH = (NJ / 2) * (NI / 4);  // phases per K step, 16 MFMAs each (4 / 2)
  constexpr int P_BYTES = BM * 128, W_BYTES = BN * 128, BUF = P_BYTES + W_BYTES;
  constexpr int NROW = BM / 64;      // 8-row pixel DMA pieces per wave per stage
  constexpr int WPIECES = BN / 64;   // weight DMA pieces per wave per stage
  constexpr int DMA_OPS = NROW + WPIECES;
  constexpr int SROWS = 2;           // statistics rows per block (one per wave row)
  constexpr int ST_OFF = NST * BUF;   // BN statistics: [SROWS][2][BN] fp32
  static_assert(NST * BUF + SROWS * 2 * BN * 4 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[NST * BUF + SROWS * 2 * BN * 4];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int gch = (lane & 7) ^ (lane >> 3);
  const int wpx = wm * 128;   // first pixel row of this wave in the tile
  const int wco = wn * WNT;   // first cout of this wave in the tile

  const uint32_t G = gridDim.x;
  const uint32_t lid = xcd_remap(blockIdx.x, G);
  const int my_tiles = lid < (uint32_t)a.ntiles ? (a.ntiles - 1 - (int)lid) / (int)G + 1 : 0;
  const int total = my_tiles * a.nks;

  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rx2 = make_rsrc(a.x2 ? a.x2 : a.x1, a.x2 ? a.xbytes2 : 0u);
  const auto rw = make_rsrc(a.w, a.wbytes);
  const auto ry1 = make_rsrc(a.y1, a.ybytes1);
  const auto ry2 = make_rsrc(a.y2 ? a.y2 : a.y1, a.y2 ? a.ybytes2 : 0u);

  // DMA state of the tile being staged (see conv_igemm_kernel::set_tile). Split-K (ksplit > 1):
  // work item = (tile, split) as in conv_igemm_kernel, K steps [ks0, ks0 + nks) of the tile.
  const int tiles1 = SPLIT ? a.ntiles / a.ksplit : a.ntiles;
  uint32_t pb1[NROW], pb2[NROW], nmask[NROW], woff[WPIECES];
  int itap = 0, icc = 0;
  auto set_tile = [&](int t) {
    const int item = (int)lid + t * (int)G;
    const int tile = SPLIT ? item % tiles1 : item;
    const int ks0 = SPLIT ? (item / tiles1) * a.nks : 0;
    itap = ks0 / a.cpt;
    icc = ks0 - itap * a.cpt;
    const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      const int m = tm * BM + (wave * NROW + r) * 8 + (lane >> 3);
      const bool valid = m < a.M;
      const uint32_t mm = valid ? (uint32_t)m : 0u;
      const uint32_t img = (__umulhi(mm, a.fhw_m) + mm) >> a.fhw_s;
      const uint32_t hw = mm - img * (uint32_t)(a.H * a.W);
      const uint32_t h = (__umulhi(hw, a.fw_m) + hw) >> a.fw_s;
      const uint32_t w = hw - h * (uint32_t)a.W;
      if constexpr (UTR) {  // the (2h + toy, 2w + tox) pixel of the output-gradient map; 4 valid taps
        const uint32_t px = (img * (uint32_t)a.tH2 + 2u * h + (uint32_t)a.toy) * (uint32_t)a.tW2 + 2u * w + (uint32_t)a.tox;
        nmask[r] = valid ? ~0xfu : ~0u;
        pb1[r] = (px * (uint32_t)a.pitch1 + (uint32_t)gch * 8u) * 2u;
        pb2[r] = pb1[r];
        continue;
      }
      const uint32_t rok = (h > 0 ? 1u : 0u) | 2u | (h + 1 < (uint32_t)a.H ? 4u : 0u);
      const uint32_t cok = (w > 0 ? 1u : 0u) | 2u | (w + 1 < (uint32_t)a.W ? 4u : 0u);
      uint32_t msk = 0;
      msk |= (rok & 1u) ? cok : 0u;
      msk |= (rok & 2u) ? (cok << 3) : 0u;
      msk |= (rok & 4u) ? (cok << 6) : 0u;
      if (a.taps == 1) msk = 1u;
      nmask[r] = valid ? ~msk : ~0u;
      pb1[r] = (mm * (uint32_t)a.pitch1 + (uint32_t)gch * 8u) * 2u;
      pb2[r] = (mm * (uint32_t)a.pitch2 + (uint32_t)gch * 8u) * 2u;
    }
#pragma unroll
    for (int f = 0; f < WPIECES; ++f) {
      const int n = tn * BN + (wave * WPIECES + f) * 8 + (lane >> 3);
      woff[f] = (uint32_t)(n * a.ldw + gch * 8 + ks0 * 64) * 2u;  // + the split's first K column
    }
  };
  auto issue = [&](int ks, char* buf) {
    const int c0 = icc * 64;
    const bool s2 = c0 >= a.C1;
    const int pitch = s2 ? a.pitch2 : a.pitch1;
    const int tap_lin = UTR ? (itap >> 1) * a.tW2 + (itap & 1) : a.taps == 9 ? tap_dr(itap) * a.W + tap_ds(itap) : 0;
    const int soff = (tap_lin * pitch + (s2 ? c0 - a.C1 : c0)) * 2;
    const int bit = UTR || a.taps == 9 ? itap : 0;
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      const uint32_t bad = __builtin_amdgcn_ubfe(nmask[r], (uint32_t)bit, 1u);
      const uint32_t off = (bad << 31) | (uint32_t)((int)(s2 ? pb2[r] : pb1[r]) + soff);
      dma16(s2 ? rx2 : rx1, (lds_void*)(buf + (wave * NROW + r) * 1024), off);
    }
    if (++icc == a.cpt) { icc = 0; ++itap; if (itap == a.taps) itap = 0; }
    char* wbuf = buf + P_BYTES;
#pragma unroll
    for (int f = 0; f < WPIECES; ++f)
      dma16(rw, (lds_void*)(wbuf + (wave * WPIECES + f) * 1024), woff[f] + (uint32_t)ks * 128u);
  };

  int rdoff[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) rdoff[hf] = (lane & 15) * 128 + 16 * (((lane >> 4) + 4 * hf) ^ (lane & 7));

  const int srow = wm;
  float* const sst = (float*)(smem + ST_OFF) + srow * 2 * BN;  // this wave (row)'s statistics words
  // UT: the bias in the (unused) statistics words, read by the epilogue with LDS loads -- a global load
  // there would wait (vmcnt) for the in-flight DMA stages too. 2^tlc <= 4 BN floats (host-checked).
  const float* const sbias = (const float*)(smem + ST_OFF);
  if constexpr (UT) {
    for (int c = (int)threadIdx.x * 4; c < (1 << a.tlc); c += 512 * 4)
      *(float4*)(smem + ST_OFF + c * 4) = *(const float4*)(a.ubias + c);
  }
  if (a.stats && (lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = wco + j * 16 + 4 * (lane >> 4);
      *(float4*)(sst + c) = make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)(sst + BN + c) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  f32x4 acc[NJ][NI];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // [cout half held][k half][cout frag of the phase] / [k half][pixel frag of the phase]
  bf16x8 fa[HOLDB ? 2 : 1][2][2], fb[2][4];

  int ks = 0, t = 0;              // compute position
  int iks = 0, it = 0, ig = 0;    // newest issued stage: K step, tile, global index
  int cbuf = 0, ibuf = 0;
  if (total > 0) {
    set_tile(0);
    issue(0, smem);
    if (NST > 2 && total > 1) {
      if (++iks == a.nks) { iks = 0; ++it; set_tile(it); }
      issue(iks, smem + BUF);
      ig = 1;
      ibuf = 1;
    }
    if (ig > 0) vm_wait<DMA_OPS>();
    else vm_wait<0>();
  }
  raw_barrier();
  if (wm == 1) raw_barrier();  // stagger the two wave groups by one segment

  auto epilogue = [&]() {
    const int item = (int)lid + t * (int)G;
    if constexpr (SPLIT) {  // fp32 partial tile -> slab[split][m][n]; conv_splitk_reduce_kernel finishes
      const int tile = item % tiles1, split = item / tiles1;
      const int tm = tile / a.tilesN, tn = tile - tm * a.tilesN;
      const auto rk = make_rsrc(a.kslab, (uint32_t)((long)a.ksplit * a.M * a.Cout * 4));
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = tn * BN + wco + j * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int m = tm * BM + wpx + i * 16 + (lane & 15);
          const uint32_t off = m < a.M ? (uint32_t)(((long)split * a.M + m) * a.Cout + n) * 4u : RDP_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j][i]), rk, off, 0, 0);
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      return;
    }
    const int tm = item / a.tilesN, tn = item - tm * a.tilesN;
    const int m0 = tm * BM, n0 = tn * BN;
    const int gq = lane >> 4;
    const int coff = 16 * (gq & 1) + 8 * (gq >> 1);
    float s1[NJ][4], s2[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int jp = 0; jp < NJ; jp += 2) {
      const int nb = n0 + wco + jp * 16;
      const int n = nb + coff;
      const bool d2 = nb >= a.Cy1;  // wave-uniform: Cy1 % 32 == 0 (host-checked), one SRD per store
      const int nn = d2 ? n - a.Cy1 : n;
      const int yp = d2 ? a.ypitch2 : a.ypitch1;
      // UT: sub-pixel of this cout pair (wave-uniform: 2^tlc >= 64) and its offset from the (2h, 2w) pixel
      const int sub = UT ? nb >> a.tlc : 0, cmask = UT ? (1 << a.tlc) - 1 : 0;
      const int subo = UT ? ((sub >> 1) * a.tW2 + (sub & 1)) * yp + (n & cmask) : 0;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int m = m0 + wpx + i * 16 + (lane & 15);
        uint2 v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = jp + h;
          f32x4 o = acc[j][i];
          if (a.escale) {
            const int nc = nb + h * 16 + 4 * gq;
            const float4 sc = *(const float4*)(a.escale + nc), sh = *(const float4*)(a.eshift + nc);
            o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
            o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
            if (a.erelu) {
              o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
            }
          } else if (UT) {
            const float4 b = *(const float4*)(sbias + ((nb + h * 16 + 4 * gq) & cmask));
            o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w;
          }
          v[h].x = pack2bf(o[0], o[1]);
          v[h].y = pack2bf(o[2], o[3]);
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (a.stats && m < a.M) {
            const float q0 = __uint_as_float(v[h].x << 16), q1 = __uint_as_float(v[h].x & 0xffff0000u);
            const float q2 = __uint_as_float(v[h].y << 16), q3 = __uint_as_float(v[h].y & 0xffff0000u);
            s1[j][0] += q0; s2[j][0] += q0 * q0;
            s1[j][1] += q1; s2[j][1] += q1 * q1;
            s1[j][2] += q2; s2[j][2] += q2 * q2;
            s1[j][3] += q3; s2[j][3] += q3 * q3;
          }
        }
        const auto rxs = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
        const auto rys = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
        uint32_t pix = (uint32_t)m * (uint32_t)yp + (uint32_t)nn;
        if constexpr (UT) {  // low-res pixel (img, h, w) -> the (2h + toy, 2w + tox) pixel of the output map
          // W % 16 == 0: the 16 pixels of fragment row i lie in one image row, so the division runs once
          // on the (wave-uniform) first pixel; else per lane
          const bool row16 = (a.W & 15) == 0;
          const uint32_t mm = row16 ? (uint32_t)(m0 + wpx + i * 16) : (uint32_t)m;
          const uint32_t img = (__umulhi(mm, a.fhw_m) + mm) >> a.fhw_s;
          const uint32_t hw = mm - img * (uint32_t)(a.H * a.W);
          const uint32_t hh = (__umulhi(hw, a.fw_m) + hw) >> a.fw_s;
          const uint32_t ww = hw - hh * (uint32_t)a.W + (row16 ? (uint32_t)(lane & 15) : 0u);
          pix = ((img * (uint32_t)a.tH2 + 2u * hh + (uint32_t)a.toy) * (uint32_t)a.tW2 + 2u * ww + (uint32_t)a.tox) *
                    (uint32_t)yp + (uint32_t)subo;
        }
        const uint32_t off = m < a.M ? pix * 2u : RDP_OOB;
        bstore16(d2 ? ry2 : ry1, off, make_uint4(rxs[0], rys[0], rxs[1], rys[1]));
      }
    }
    if (a.stats) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] = row16_sum(s1[j][r]);
          s2[j][r] = row16_sum(s2[j][r]);
        }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = wco + j * 16 + 4 * gq;
          float4 u = *(float4*)(sst + c), q = *(float4*)(sst + BN + c);
          u.x += s1[j][0]; u.y += s1[j][1]; u.z += s1[j][2]; u.w += s1[j][3];
          q.x += s2[j][0]; q.y += s2[j][1]; q.z += s2[j][2]; q.w += s2[j][3];
          *(float4*)(sst + c) = u;
          *(float4*)(sst + BN + c) = q;
        }
      }
    }
  };

  for (int g = 0; g < total; ++g) {
    const char* pb = smem + cbuf * BUF;
    const char* wb = pb + P_BYTES;
#pragma unroll
    for (int p = 0; p < NPH; ++p) {
      // phase -> (pixel half ih, cout half jh): BN 256: (0,0) (0,1) (1,1) (1,0); BN 128: (0,*) (1,*)
      const int ih = NPH == 4 ? (p >> 1) : p;
      const int jh = NPH == 4 ? (((p + 1) >> 1) & 1) : 0;
      const bool new_b = NPH == 4 ? (p == 0 || p == 2) : true;
      const bool new_a = NPH == 4 ? (HOLDB ? p < 2 : p != 2) : (p == 0);
      const int fh = HOLDB ? jh : 0;  // register set of the phase's weight fragments
      // ---- memory segment
      if (p == 0 && ig + 1 < total) {
        if (++iks == a.nks) { iks = 0; ++it; set_tile(it); }
        ibuf = ibuf + 1 == NST ? 0 : ibuf + 1;
        issue(iks, smem + ibuf * BUF);
        ++ig;
      }
      if (new_a) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int j = 0; j < 2; ++j) fa[fh][hf][j] = *(const bf16x8*)(wb + (wco / 16 + jh * 2 + j) * 2048 + rdoff[hf]);
      }
      if (new_b) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int i = 0; i < 4; ++i) fb[hf][i] = *(const bf16x8*)(pb + (wpx / 16 + ih * 4 + i) * 2048 + rdoff[hf]);
      }
      // The last memory segment of a K step drains its fragment reads (lgkmcnt(0)) before the barrier:
      // the next DMA into this buffer follows that barrier (WAR). The other phases' reads stay in
      // flight across the barrier and are waited for by the MFMAs that use them (the segment ends as
      // soon as they are issued; their LDS latency overlaps the partner group's MFMA cluster).
      if (p == NPH - 1 && g + 1 < total) {  // + this wave's DMA of stage g+1 has landed
        if (ig > g + 1) vm_wait<DMA_OPS>();
        else vm_wait<0>();
      } else if (p == NPH - 1 || !RD_INFLIGHT) {
        wait_lgkm0();
      }
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- compute segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[jh * 2 + j][ih * 4 + i] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[fh][hf][j], fb[hf][i], acc[jh * 2 + j][ih * 4 + i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (p == NPH - 1 && ks + 1 == a.nks) epilogue();
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
    }
    cbuf = cbuf + 1 == NST ? 0 : cbuf + 1;
    if (++ks == a.nks) { ks = 0; ++t; }
  }
  if (wm == 0) raw_barrier();  // same barrier count for both groups
  if (a.stats && total > 0 && (lane & 15) == 0) {
    const int tn = (int)lid % a.tilesN;
    float* row = a.stats + (size_t)(((int)lid / a.tilesN) * SROWS + srow) * 2 * a.Cout;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wco + j * 16 + 4 * (lane >> 4);
      *(float4*)(row + tn * BN + cl) = *(const float4*)(sst + cl);
      *(float4*)(row + a.Cout + tn * BN + cl) = *(const float4*)(sst + BN + cl);
    }
  }
}

static int launch_split_reduce(const ConvArgs& a, hipStream_t s, int* pooled);

// ksplit > 1 (a.kslab set, ksplit divides nks, slab within 2 GiB -- the caller's plan): fp32
// partial tiles, then the shared split-K reduce (stats / eval epilogue / fused pool or upsample).
template <int BN>
static int launch_pp(ConvArgs a, hipStream_t s, int ksplit = 1, int* pooled = nullptr) {
  constexpr int BM = 256;
  if (a.packed || a.Cout % BN || a.Cy1 % 32) return -1;
  const int tilesM = (a.M + BM - 1) / BM;
  a.tilesN = a.Cout / BN;
  a.ntiles = tilesM * a.tilesN;
  if (ksplit > 1) {
    if (!a.kslab || a.nks % ksplit) return -1;
    a.ksplit = ksplit;
    a.nks /= ksplit;
    a.ntiles *= ksplit;
    ConvArgs k = a;
    k.stats = nullptr;  // statistics come from the reduce
    const int grid = k.ntiles < 256 ? k.ntiles : 256;
    hipLaunchKernelGGL((conv_pp_kernel<BN, true>), dim3(grid), dim3(512), 0, s, k);
    return launch_split_reduce(a, s, pooled);
  }
  a.ksplit = 1;
  a.pool = nullptr;
  a.up = nullptr;
  if (a.tlc || a.taps == 4) {  // ConvTranspose2d output (rdp_conv_upT_fwd) / input gradient (rdp_conv_upT_dgrad)
    if (a.stats || a.escale || a.y2) return -1;
    const int grid = a.ntiles < 256 ? a.ntiles : 256;
    if (a.tlc) hipLaunchKernelGGL((conv_pp_kernel<BN, false, true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv_pp_kernel<BN, false, false, true>), dim3(grid), dim3(512), 0, s, a);
    return 0;
  }
  // one persistent block per CU (512 blocks or one block per tile, which let the dispatcher balance
  // the tiles around the concurrent wgrads, measured 0.8 % / 1.7 % slower: profiles/dead_ends.md)
  const int grid = a.ntiles < 256 ? a.ntiles : 256;
  if (a.stats && grid % a.tilesN) return -1;
  hipLaunchKernelGGL((conv_pp_kernel<BN>), dim3(grid), dim3(512), 0, s, a);
  return grid / a.tilesN * 2;
}

// ConvTranspose2d(k=2, s=2) + bias straight into its (padded) output map u [N][H2][W2][upitch]: the
// 1x1 GEMM yT[px][sub * C + c] = sum_ci x[px][ci] Wt[sub * C + c][ci] on the ping-pong kernel with the
// sub-pixel scatter + bias in its epilogue (no yT round trip and no upT_shuffle pass). u's border
// outside the 2h x 2w window at (oy, ox) is not written (the caller zeroes it once). Returns 0, or -1
// where the ping-pong grid would not fill the chip / the shape does not fit (the caller then runs the
// GEMM + upT_shuffle).
extern "C" int rdp_conv_upT_fwd(const void* x, long xbytes, int Cin, int pitch, const void* w, long wbytes, int ldw,
                                void* u, long ubytes, int upitch, const float* bias, int N, int h, int wd, int H2,
                                int W2, int oy, int ox, int C, hipStream_t s) {
  // (C <= 512: the bias fits the kernel's 4 BN statistics words at BN = 128)
  if (C < 64 || C > 512 || (C & (C - 1)) || Cin % 64 || ldw < Cin || upitch % 8 || oy < 0 || ox < 0 ||
      2 * h + oy > H2 || 2 * wd + ox > W2)
    return -1;
  if (xbytes >= (1l << 31) || ubytes >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  ConvArgs a;
  a.x1 = (const u16*)x; a.x2 = nullptr; a.xbytes1 = (uint32_t)xbytes; a.xbytes2 = 0;
  a.C1 = Cin; a.C2 = 0; a.pitch1 = pitch; a.pitch2 = pitch;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y1 = (u16*)u; a.y2 = nullptr; a.ybytes1 = (uint32_t)ubytes; a.ybytes2 = 0;
  a.Cout = 4 * C; a.Cy1 = a.Cout; a.ypitch1 = upitch; a.ypitch2 = upitch; a.stats = nullptr;
  a.escale = nullptr; a.eshift = nullptr; a.erelu = 0;
  a.N = N; a.H = h; a.W = wd; a.M = N * h * wd;
  a.taps = 1; a.packed = 0; a.cpt = Cin / 64; a.nks = a.cpt;
  a.ksplit = 1; a.kslab = nullptr; a.pool = nullptr; a.up = nullptr;
  const FastDiv fhw = make_fastdiv((uint32_t)(h * wd)), fw = make_fastdiv((uint32_t)wd);
  a.fhw_m = fhw.m; a.fhw_s = fhw.s; a.fw_m = fw.m; a.fw_s = fw.s;
  a.ubias = bias; a.tH2 = H2; a.tW2 = W2; a.toy = oy; a.tox = ox;
  a.tlc = 0;
  while ((1 << a.tlc) < C) ++a.tlc;
  if (a.Cout % 256 == 0 && (long)(a.M + 255) / 256 * (a.Cout / 256) >= 256) return launch_pp<256>(a, s) >= 0 ? 0 : -1;
  if (Cin >= 128 && (long)(a.M + 255) / 256 * (a.Cout / 128) >= 256) return launch_pp<128>(a, s) >= 0 ? 0 : -1;
  return -1;
}

// ConvTranspose2d(k=2, s=2) input gradient straight from the output gradient du [N][H2][W2][C] (the
// window 2h x 2w at (oy, ox)): dx[px][ci] = sum_(sub, c) du[sub-pixel sub of px][c] Wd[ci][sub * C + c]
// on the ping-pong kernel, its A operand DMA'd from the 4 sub-pixels as 4 "taps" (no unshuffled copy
// of du). wd = the [Cin][4C] dgrad weight. Returns 0, or -1 where the ping-pong grid would not fill
// the chip / the shape does not fit (the caller unshuffles and runs the 1x1 GEMM).
extern "C" int rdp_conv_upT_dgrad(const void* du, long dubytes, int C, int dupitch, int H2, int W2, int oy, int ox,
                                  const void* wd, long wbytes, int ldw, void* dx, long dxbytes, int Cin, int dxpitch,
                                  int N, int h, int wdt, hipStream_t s) {
  if (C % 64 || Cin % 128 || ldw < 4 * C || oy < 0 || ox < 0 || 2 * h + oy > H2 || 2 * wdt + ox > W2) return -1;
  if (dubytes >= (1l << 31) || dxbytes >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  ConvArgs a;
  a.x1 = (const u16*)du; a.x2 = nullptr; a.xbytes1 = (uint32_t)dubytes; a.xbytes2 = 0;
  a.C1 = C; a.C2 = 0; a.pitch1 = dupitch; a.pitch2 = dupitch;
  a.w = (const u16*)wd; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y1 = (u16*)dx; a.y2 = nullptr; a.ybytes1 = (uint32_t)dxbytes; a.ybytes2 = 0;
  a.Cout = Cin; a.Cy1 = Cin; a.ypitch1 = dxpitch; a.ypitch2 = dxpitch; a.stats = nullptr;
  a.escale = nullptr; a.eshift = nullptr; a.erelu = 0;
  a.N = N; a.H = h; a.W = wdt; a.M = N * h * wdt;
  a.taps = 4; a.packed = 0; a.cpt = C / 64; a.nks = 4 * a.cpt;
  a.ksplit = 1; a.kslab = nullptr; a.pool = nullptr; a.up = nullptr;
  const FastDiv fhw = make_fastdiv((uint32_t)(h * wdt)), fw = make_fastdiv((uint32_t)wdt);
  a.fhw_m = fhw.m; a.fhw_s = fhw.s; a.fw_m = fw.m; a.fw_s = fw.s;
  a.tH2 = H2; a.tW2 = W2; a.toy = oy; a.tox = ox;
  if (Cin % 256 == 0 && (long)(a.M + 255) / 256 * (Cin / 256) >= 256) return launch_pp<256>(a, s) >= 0 ? 0 : -1;
  if ((long)(a.M + 255) / 256 * (Cin / 128) >= 256) return launch_pp<128>(a, s) >= 0 ? 0 : -1;
  return -1;
}

extern "C" int rdp_conv_ring(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                             void* y, long ybytes, int ypitch, void* y2, long ybytes2, int ypitch2, int Cy1,
                             int Cout, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                             int erelu, int max_blocks, hipStream_t s);
extern "C" int rdp_conv_ring_pool(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                                  void* y, long ybytes, int ypitch, int Cout, int N, int H, int W,
                                  const float* escale, const float* eshift, int erelu, void* pool, int ppitch,
                                  hipStream_t s);
extern "C" int rdp_conv_halo_tiles(int N, int H, int W, int C1, int C2, int Cout, int taps, int packed);
extern "C" int rdp_conv_rowband(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2, int pitch1,
                                int pitch2, const void* w, long wbytes, int ldw, void* y, long ybytes, int ypitch, int N,
                                int H, int W, int Cout, const float* escale, const float* eshift, int erelu, void* pool,
                                long pbytes, int ppitch, hipStream_t s);

extern "C" long rdp_conv_rowband_bytes(int N, int H, int W, int Cin, int Cout, int pool);

// Eval convs on small maps run on the row-band kernel (csrc/conv_rowband.hip) where its operand traffic
// model says it wins (<= 160 MB; a pool it cannot fuse would cost a separate launch): RDP_ROWBAND=0 turns
// the auto choice off (A/B); bm_pref 16 forces it.
static bool rowband_auto(int N, int H, int W, int Cin, int Cout, bool pool) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("RDP_ROWBAND");
    on = e ? atoi(e) : 1;
  }
  if (on == 0 || (long)N * H * W > 4096 || W > 64 || Cin < 128 || Cout < 64) return false;
  if (pool && !(H % 2 == 0 && 2 * W <= 64)) return false;
  // (the estimate without the pool's two-row blocks: with or without a pool the same kernel runs, so the
  // two calls give bitwise the same activations)
  return rdp_conv_rowband_bytes(N, H, W, Cin, Cout, 0) <= 160000000L;
}
extern "C" int rdp_conv_ring2(const void* x0, long xbytes0, int pitch0, const void* x1, long xbytes1, int pitch1,
                              const void* w, long wbytes, int ldw, void* y, long ybytes, int ypitch, float* stats,
                              int N, int H, int W, const float* escale, const float* eshift, int erelu, int max_blocks,
                              int cout_total, int co0, hipStream_t s);
extern "C" int rdp_conv_first(const void* x, long xbytes, int pitch, const void* w, long wbytes, void* y, long ybytes,
                              int ypitch, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                              int erelu, hipStream_t s);
extern "C" int rdp_conv_halo(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2, int pitch1,
                             int pitch2, const void* w, long wbytes, int ldw, void* y1, void* y2, long ybytes1,
                             long ybytes2, int Cy1, int ypitch1, int ypitch2, float* stats, int N, int H, int W,
                             int Cout, const float* escale, const float* eshift, int erelu, hipStream_t s);

// Split-K reduction + epilogue: y[m][n] = epi(sum_s slab[s][m][n]); optional BN-stats rows (one per
// block). Thread = fixed 4-channel group (epilogue coefficients in registers), rows grid-strided.
// The slices are read 8 at a time as independent 16-B buffer loads (slices past ksplit read zeros
// from an out-of-range offset: no branch around the loads) into 4 accumulators summed in a fixed
// order: a dependent load per slice made this kernel one L2 round trip per slice (7-8 us at 18
// slices at N = 1; the serving convs reduce 2-18 slices).
__global__ __launch_bounds__(256) void conv_splitk_reduce_kernel(const ConvArgs a, int nrow_blocks) {
  extern __shared__ float sst[];  // [rows][2][Cout] stats staging
  const int CG = a.Cout >> 2, RPB = 256 / CG;  // Cout power of two, 64 <= Cout <= 1024
  const int g = threadIdx.x & (CG - 1), r = threadIdx.x / CG;
  const int n = g * 4;
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.escale) sc = *(const float4*)(a.escale + n);
  if (a.eshift) sh = *(const float4*)(a.eshift + n);
  const bool d2 = n >= a.Cy1;
  const int nn = d2 ? n - a.Cy1 : n;
  u16* const y = d2 ? a.y2 : a.y1;
  const int yp = d2 ? a.ypitch2 : a.ypitch1;
  const auto rk = make_rsrc(a.kslab, (uint32_t)((long)a.ksplit * a.M * a.Cout * 4));
  const uint32_t sstride = (uint32_t)a.M * (uint32_t)a.Cout * 4u;  // bytes between slices
  f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
  // sum of the slices + epilogue for pixel m -> 4 bf16 (packed), stored to y
  auto pixel = [&](int m) -> uint2 {
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t base = ((uint32_t)m * (uint32_t)a.Cout + (uint32_t)n) * 4u;
    for (int sp0 = 0; sp0 < a.ksplit; sp0 += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t off = sp0 + u < a.ksplit ? base + (uint32_t)(sp0 + u) * sstride : RDP_OOB;
        v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u & 3] += v[u];
    }
    f32x4 o = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
    o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
    if (a.erelu) {
      o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
    }
    const uint2 w = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    *(uint2*)(y + (long)m * yp + nn) = w;
    return w;
  };
  if (a.pool) {
    // eval-mode MaxPool2d(2) of the output, fused: a thread owns 2x2 windows (H, W even)
    const int Ho = a.H >> 1, Wo = a.W >> 1, nwin = a.M >> 2;
    for (int wi = blockIdx.x * RPB + r; wi < nwin; wi += nrow_blocks * RPB) {
      const int img = wi / (Ho * Wo), rem = wi - img * (Ho * Wo), ho = rem / Wo, wo = rem - ho * Wo;
      const int m00 = (img * a.H + 2 * ho) * a.W + 2 * wo;
      const uint2 q[4] = {pixel(m00), pixel(m00 + 1), pixel(m00 + a.W), pixel(m00 + a.W + 1)};
      float mx[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t wd = k < 2 ? q[0].x : q[0].y;
        mx[k] = __uint_as_float((k & 1) ? (wd & 0xffff0000u) : (wd << 16));
      }
#pragma unroll
      for (int t = 1; t < 4; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t wd = k < 2 ? q[t].x : q[t].y;
          mx[k] = fmaxf(mx[k], __uint_as_float((k & 1) ? (wd & 0xffff0000u) : (wd << 16)));
        }
      *(uint2*)(a.pool + (long)wi * a.ppitch + n) = make_uint2(pack2bf(mx[0], mx[1]), pack2bf(mx[2], mx[3]));
    }
    return;  // eval: no statistics
  }
  // BN-backward partials (a.bnpart): the owner layer's coefficients of this thread's 4 channels
  const bool bnr = a.stats == nullptr && a.bnpart != nullptr;
  float bmean[4], binv[4], bsc[4], bsh[4];
  if (bnr) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bmean[k] = a.bncoef[n + k];
      binv[k] = a.bncoef[a.Cout + n + k];
      bsc[k] = a.bncoef[2 * a.Cout + n + k];
      bsh[k] = a.bncoef[3 * a.Cout + n + k];
    }
  }
  for (int m = blockIdx.x * RPB + r; m < a.M; m += nrow_blocks * RPB) {
    const uint2 w = pixel(m);
    const float q[4] = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                        __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
    if (a.stats) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { s1[k] += q[k]; s2[k] += q[k] * q[k]; }
    } else if (bnr) {  // q = dL/da (as stored, bf16) of the owner's post-ReLU activation
      const uint2 yv = *(const uint2*)(a.bny + (long)m * a.bnypitch + n);
      const float fy[4] = {__uint_as_float(yv.x << 16), __uint_as_float(yv.x & 0xffff0000u),
                           __uint_as_float(yv.y << 16), __uint_as_float(yv.y & 0xffff0000u)};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float g = fmaf(fy[k], bsc[k], bsh[k]) > 0.f ? q[k] : 0.f;
        s1[k] += g;
        s2[k] += g * (fy[k] - bmean[k]) * binv[k];
      }
    }
  }
  float* const rows_out = a.stats ? a.stats : (bnr ? a.bnpart : nullptr);
  if (!rows_out) return;
  *(float4*)(sst + (r * 2 + 0) * a.Cout + n) = make_float4(s1[0], s1[1], s1[2], s1[3]);
  *(float4*)(sst + (r * 2 + 1) * a.Cout + n) = make_float4(s2[0], s2[1], s2[2], s2[3]);
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * a.Cout; c += 256) {
    const int half = c / a.Cout, ch = c - half * a.Cout;
    float acc = 0.f;
    for (int qq = 0; qq < RPB; ++qq) acc += sst[(qq * 2 + half) * a.Cout + ch];
    rows_out[(long)blockIdx.x * 2 * a.Cout + c] = acc;
  }
}

// Split-K reduce fused with the decoder's bilinear x2 upsample (eval; serving at N = 1): a block owns
// UP_TY output rows of one image x UP_CG channels. Phase 1 reduces the slices of the (at most
// UP_TY / 2 + 2) source rows those output rows read -- same summation and epilogue as
// conv_splitk_reduce_kernel, so the low-resolution output y is written bitwise as there (rows shared by
// two bands are written twice with equal values) -- into LDS as bf16; phase 2 interpolates the output
// rows from LDS with the arithmetic of upsample2_fwd_kernel (csrc/pool_up.hip). The low-res tensor is
// never re-read from memory and the upsample launch disappears.
#define UP_TY 4
#define UP_CG 16
RDP_DEV void up_src_f(int u, int in, float r, int& i0, int& i1, float& l1) {  // = up_src (pool_up.hip)
  const float sv = r * (float)u;
  i0 = (int)sv;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = sv - (float)i0;
}
__global__ __launch_bounds__(256) void conv_splitk_reduce_up_kernel(const ConvArgs a) {
  extern __shared__ uint32_t srcs[];  // [source row][W][UP_CG / 2] packed bf16 pairs
  const int nb = (a.uH + UP_TY - 1) / UP_TY;
  const int img = blockIdx.x / nb, band = blockIdx.x - img * nb;
  const int c0 = blockIdx.y * UP_CG;
  const int Y0 = band * UP_TY, Y1 = min(a.uH, Y0 + UP_TY);
  int sy_lo = a.H, sy_hi = -1;
  for (int Y = Y0; Y < Y1; ++Y) {
    const int uy = Y - a.uoy;
    if (uy < 0 || uy >= 2 * a.H) continue;
    int y0, y1;
    float ly;
    up_src_f(uy, a.H, a.urh, y0, y1, ly);
    sy_lo = min(sy_lo, y0);
    sy_hi = max(sy_hi, y1);
  }
  const int nrows = sy_hi >= sy_lo ? sy_hi - sy_lo + 1 : 0;
  const auto rk = make_rsrc(a.kslab, (uint32_t)((long)a.ksplit * a.M * a.Cout * 4));
  const uint32_t sstride = (uint32_t)a.M * (uint32_t)a.Cout * 4u;
  constexpr int NQ = UP_CG / 4;  // 4-channel quads per block
  for (int it = threadIdx.x; it < nrows * a.W * NQ; it += 256) {
    const int q = it % NQ, px = it / NQ;
    const int r = px / a.W, x = px - r * a.W;
    const int m = (img * a.H + sy_lo + r) * a.W + x;
    const int n = c0 + 4 * q;
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t base = ((uint32_t)m * (uint32_t)a.Cout + (uint32_t)n) * 4u;
    for (int sp0 = 0; sp0 < a.ksplit; sp0 += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t off = sp0 + u < a.ksplit ? base + (uint32_t)(sp0 + u) * sstride : RDP_OOB;
        v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u & 3] += v[u];
    }
    f32x4 o = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const float4 sc = *(const float4*)(a.escale + n), sh = *(const float4*)(a.eshift + n);
    o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
    o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
    if (a.erelu) {
      o[0] = fmaxf(o[0], 0.f); o[1] = fmaxf(o[1], 0.f); o[2] = fmaxf(o[2], 0.f); o[3] = fmaxf(o[3], 0.f);
    }
    const uint2 w = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    *(uint2*)(a.y1 + (long)m * a.ypitch1 + n) = w;
    srcs[(px * NQ + q) * 2] = w.x;
    srcs[(px * NQ + q) * 2 + 1] = w.y;
  }
  __syncthreads();
  for (int it = threadIdx.x; it < (Y1 - Y0) * a.uW * NQ; it += 256) {
    const int q = it % NQ, t = it / NQ;
    const int X = t % a.uW, Y = Y0 + t / a.uW;
    const int uy = Y - a.uoy, ux = X - a.uox;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (!(uy < 0 || ux < 0 || uy >= 2 * a.H || ux >= 2 * a.W)) {
      int y0, y1, x0, x1;
      float ly, lx;
      up_src_f(uy, a.H, a.urh, y0, y1, ly);
      up_src_f(ux, a.W, a.urw, x0, x1, lx);
      auto ld = [&](int yy, int xx, float* f) {
        const int i = (((yy - sy_lo) * a.W + xx) * NQ + q) * 2;
        const uint32_t lo = srcs[i], hi = srcs[i + 1];
        f[0] = __uint_as_float(lo << 16); f[1] = __uint_as_float(lo & 0xffff0000u);
        f[2] = __uint_as_float(hi << 16); f[3] = __uint_as_float(hi & 0xffff0000u);
      };
      float pa[4], pb[4], pc[4], pd[4];
      ld(y0, x0, pa); ld(y0, x1, pb); ld(y1, x0, pc); ld(y1, x1, pd);
      const float hy = 1.f - ly, hx = 1.f - lx;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = hy * (hx * pa[k] + lx * pb[k]) + ly * (hx * pc[k] + lx * pd[k]);
    }
    *(uint2*)(a.up + ((long)(img * a.uH + Y) * a.uW + X) * a.upitch + c0 + 4 * q) =
        make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
  }
}

// The reduce + epilogue launch after a split-K conv: returns the stats rows written (0 with the fused
// upsample / pool, whose *pooled is set)
static int launch_split_reduce(const ConvArgs& a, hipStream_t s, int* pooled) {
  const int rpb = 256 / (a.Cout / 4);
  int nblk = (a.M + rpb - 1) / rpb;  // <= 512 stats rows: within conv_stats_rows()'s bound
  nblk = nblk < 512 ? nblk : 512;
  if (a.up) {  // fused eval upsample: bands of UP_TY output rows x UP_CG channels
    const int nb = (a.uH + UP_TY - 1) / UP_TY;
    const size_t lds = (size_t)(UP_TY / 2 + 2) * a.W * UP_CG * 2;
    hipLaunchKernelGGL(conv_splitk_reduce_up_kernel, dim3(a.N * nb, a.Cout / UP_CG), dim3(256), lds, s, a);
    if (pooled) *pooled = 1;
    return 0;
  }
  if (a.pool) {  // fused eval MaxPool2d(2): one work row per 2x2 window, no stats rows
    nblk = (a.M / 4 + rpb - 1) / rpb;
    nblk = nblk < 2048 ? nblk : 2048;
    if (pooled) *pooled = 1;
  }
  const bool bnr = !a.stats && a.bnpart && !a.pool;
  const size_t lds = (a.stats || bnr) ? (size_t)rpb * 2 * a.Cout * sizeof(float) : 0;
  hipLaunchKernelGGL(conv_splitk_reduce_kernel, dim3(nblk), dim3(256), lds, s, a, nblk);
  if (bnr && a.bnrows) *a.bnrows = nblk;
  return nblk;
}

// Split-K when the tile grid leaves most CUs idle: the smallest divisor of the K steps that gives
// >= 256 work items with >= 4 K steps each, as long as the fp32 slab fits `ws_elems`.
static int choose_ksplit(int ntiles, int nks, int M, int Cout, int packed, long ws_elems) {
  const bool pow2 = Cout >= 64 && Cout <= 1024 && (Cout & (Cout - 1)) == 0;  // reduce kernel's groups
  int ks = 1;
  if (!pow2 || packed || ntiles >= 192) return 1;
  for (int d = 2; d <= nks / 4; ++d) {
    if (nks % d) continue;
    if ((long)d * M * Cout > ws_elems) break;
    ks = d;
    if (ntiles * d >= 256) break;
  }
  return ks;
}

// Split-K ping-pong plan for the small-M / long-K convs (reference-batch training, deep layers): the
// 256 x BN tile grid alone leaves most CUs idle, so the K steps are split over d work items (the
// smallest divisor of nks giving >= 256 items, one block per CU, each >= PP_SPLIT_MIN_KS K steps)
// when the fp32 slab d * M * Cout fits. Returns d (0: no split-K ping-pong plan).
constexpr int PP_SPLIT_MIN_KS = 8;
static int pp_split_plan(int M, int Cout, int BN, int nks, long ws_elems) {
  // (the split-K reduce kernel maps a power-of-two channel count, 64..1024, onto its threads)
  if (Cout % BN || Cout > 1024 || (Cout & (Cout - 1))) return 0;
  const long tiles = (long)(M + 255) / 256 * (Cout / BN);
  if (tiles >= 256) return 0;
  for (int d = 2; d <= nks / PP_SPLIT_MIN_KS; ++d) {
    if (nks % d) continue;
    if ((long)d * M * Cout > ws_elems) return 0;
    if (tiles * d >= 256) return d;
  }
  return 0;
}

static bool pp_split_enabled() {  // RDP_PP_SPLIT=0: the 128 x 128 split-K kernel instead (A/B)
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("RDP_PP_SPLIT");
    on = e ? atoi(e) != 0 : 1;
  }
  return on != 0;
}

template <int BM, int BN, int NWV = 4>
static int launch_cfg(ConvArgs a, int max_blocks, long ws_elems, hipStream_t s, int* pooled = nullptr) {
  const int tilesM = (a.M + BM - 1) / BM;
  a.tilesN = a.Cout / BN;
  a.ntiles = tilesM * a.tilesN;
  a.ksplit = a.kslab ? choose_ksplit(a.ntiles, a.nks, a.M, a.Cout, a.packed, ws_elems) : 1;
  if (a.ksplit > 1) {
    a.nks /= a.ksplit;
    a.ntiles *= a.ksplit;
    const int grid = a.ntiles < max_blocks ? a.ntiles : max_blocks;
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, NWV>), dim3(grid), dim3(64 * NWV), 0, s, a);
    return launch_split_reduce(a, s, pooled);
  }
  a.pool = nullptr;  // the non-split epilogue does not pool / upsample (the caller launches them)
  a.up = nullptr;
  const int grid = a.ntiles < max_blocks ? a.ntiles : max_blocks;
  // the per-block stats rows need every block to keep one channel tile (see the kernel)
  if (a.stats && grid % a.tilesN) return -1;
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, NWV>), dim3(grid), dim3(64 * NWV), 0, s, a);
  return grid / a.tilesN * (BM / 64);
}

// Returns the number of stats-slab rows written, or -1 on unsupported shape.
extern "C" int rdp_conv_igemm(const void* x1, const void* x2, long xbytes1, long xbytes2, int C1, int C2,
                              int pitch1, int pitch2, const void* w, long wbytes, int ldw, void* y1, void* y2,
                              long ybytes1, long ybytes2, int Cy1, int ypitch1, int ypitch2, float* stats,
                              int N, int H, int W, int Cout, int taps, int packed, int bm_pref,
                              const float* escale, const float* eshift, int erelu, float* ws, long ws_elems,
                              void* pool, int ppitch, int* pooled, void* up, int upitch, int uH, int uW,
                              int uoy, int uox, const void* bny, int bnypitch, const float* bncoef, float* bnpart,
                              int* bnrows, hipStream_t s) {
  // pool (eval, optional): MaxPool2d(2) of y1 fused into the split-K reduce when that path runs;
  // up (eval, optional, exclusive with pool): bilinear x2 upsample of y1 into up [N][uH][uW] at
  // (uoy, uox), fused the same way; *pooled = 1 if the fused output was written (else the caller
  // launches the pool / upsample)
  // bny / bncoef / bnpart (training dgrad into one BN + ReLU layer's activation gradient, optional): that
  // layer's BN-backward partial rows, written by the split-K reduce when that path runs (ConvArgs);
  // *bnrows = the rows written, else 0 (the caller runs bn_relu_bwd_reduce)
  if (pooled) *pooled = 0;
  if (bnrows) *bnrows = 0;
  // first layer (3-channel input, packed K): conv_first.hip (auto, or bm_pref 13 = force; bm_pref 256
  // runs this file's packed implicit GEMM, the tests' second opinion)
  {
    const int pref = bm_pref % 1000;
    if (packed && (pref == 13 || pref == 0) && C1 == 8 && C2 == 0 && x2 == nullptr && taps == 9 &&
        Cout == 64 && y2 == nullptr) {
      const int r = rdp_conv_first(x1, xbytes1, pitch1, w, wbytes, y1, ybytes1, ypitch1, stats, N, H, W, escale, eshift,
                                   erelu, s);
      if (r >= 0 || pref == 13) return r;
    }
  }
  // eval (BN folded, one destination) on small maps: the row-band kernel, MaxPool2d fused (16 = force)
  {
    const int pref = bm_pref % 1000;
    if (escale && eshift && !stats && !y2 && taps == 9 && !packed &&
        (pref == 16 || (pref == 0 && rowband_auto(N, H, W, C1 + C2, Cout, pool && pooled)))) {
      const bool wp = pool && pooled && H % 2 == 0 && W % 2 == 0;
      const long pbytes = wp ? ((long)N * (H / 2) * (W / 2) - 1) * ppitch * 2 + (long)Cout * 2 : 0;
      const int r = rdp_conv_rowband(x1, x2, xbytes1, xbytes2, C1, C2, pitch1, pitch2, w, wbytes, ldw, y1, ybytes1,
                                     ypitch1, N, H, W, Cout, escale, eshift, erelu, wp ? pool : nullptr, pbytes,
                                     ppitch, s);
      if (r >= 0) {
        if (r == 1) *pooled = 1;
        return 0;
      }
      if (pref == 16) return -1;
    }
  }
  // bm_pref % 1000: 0 = auto, 1 = force the halo-tile kernel, 6 = force the row-ring kernel,
  // 128 / 256 (2 / 3: 8-wave) = force this kernel's tile
  {
    const int pref = bm_pref % 1000;
    // row-ring kernel (conv_ring.hip): 64 -> 64 channels, 3x3, one source, no output split. Auto only
    // when its grid (one block per pair of 64-pixel row segments, <= 256) fills the chip: at N = 1,
    // 128^2 x 64 -> 128 the 128-block ring took 15.2 us vs 11.9 us for the implicit GEMM
    const long ring_pairs = W % 64 == 0 ? (long)N * (W / 64) * H / 2 : 0;
    if ((pref == 6 || (pref == 0 && ring_pairs >= 256)) && taps == 9 && !packed && C2 == 0 &&
        x2 == nullptr) {
      if (pool && pooled && !stats && !y2 && escale) {  // eval: MaxPool2d fused into the ring epilogue
        const int r = rdp_conv_ring_pool(x1, xbytes1, C1, pitch1, w, wbytes, ldw, y1, ybytes1, ypitch1, Cout, N, H, W,
                                         escale, eshift, erelu, pool, ppitch, s);
        if (r == 0) {
          *pooled = 1;
          return 0;
        }
      }
      const int r = rdp_conv_ring(x1, xbytes1, C1, pitch1, w, wbytes, ldw, y1, ybytes1, ypitch1, y2, ybytes2,
                                  ypitch2, Cy1, Cout, stats, N, H, W, escale, eshift, erelu, 256, s);
      if (r >= 0 || pref == 6) return r;
    }
  }
  // two-source row ring (conv_ring.hip conv_ring2_kernel): 128 input channels (two 64-channel sources,
  // or one 128-channel tensor as its two halves) -> 64, 3x3, one destination; 14 = force. 15 = force
  // (auto: RING2_X2_PAIRS) 128 -> 128 as two launches over the output-channel halves (each reads the input).
  {
    const int pref = bm_pref % 1000;
    const long ring_pairs = W % 64 == 0 ? (long)N * (W / 64) * H / 2 : 0;
    const bool two = C1 == 64 && C2 == 64 && x2 != nullptr, one = C1 == 128 && C2 == 0 && x2 == nullptr;
    const bool c64 = Cout == 64 && (pref == 14 || (pref == 0 && ring_pairs >= 256));
    const bool c128 = Cout == 128 && (pref == 15 || (pref == 0 && ring_pairs >= RING2_X2_PAIRS));
    if ((c64 || c128) && taps == 9 && !packed && (two || one) && y2 == nullptr && !(pool && pooled) &&
        !(up && pooled)) {
      const void* s1 = two ? x2 : (const void*)((const u16*)x1 + 64);
      const long b1 = two ? xbytes2 : xbytes1 - 128;
      int r = -1;
      for (int co0 = 0; co0 < Cout; co0 += 64) {
        const long yoff = (long)co0 * 2;
        r = rdp_conv_ring2(x1, xbytes1, pitch1, s1, b1, two ? pitch2 : pitch1, (const u16*)w + (long)co0 * ldw,
                           wbytes - (long)co0 * ldw * 2, ldw, (u16*)y1 + co0, ybytes1 - yoff, ypitch1, stats, N, H, W,
                           escale ? escale + co0 : nullptr, eshift ? eshift + co0 : nullptr, erelu, 256, Cout, co0, s);
        if (r < 0) break;
      }
      if (r >= 0 || pref == 14 || pref == 15) return r;
    }
  }
  {
    const int pref = bm_pref % 1000;
    const int ht = rdp_conv_halo_tiles(N, H, W, C1, C2, Cout, taps, packed);
    // auto: the halo kernel wins only where a 64-channel output reads >= 256 input channels
    // (measured, scripts/conv_microbench.py); elsewhere this kernel's 2 blocks/CU overlap better
    const bool halo_auto = pref == 0 && ht >= 256 && Cout == 64 && C1 + C2 >= 256;
    if (ht > 0 && (pref == 1 || halo_auto))
      return rdp_conv_halo(x1, x2, xbytes1, xbytes2, C1, C2, pitch1, pitch2, w, wbytes, ldw, y1, y2, ybytes1,
                           ybytes2, Cy1, ypitch1, ypitch2, stats, N, H, W, Cout, escale, eshift, erelu, s);
    if (pref == 1) return -1;
  }
  ConvArgs a;
  a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  // ws = the split-K fp32 slab (rdp_conv_ws_elems)
  const bool has_ws = ws != nullptr && ws_elems > 0;
  a.kslab = has_ws ? ws : nullptr;
  a.ksplit = 1;
  a.pool = (pool != nullptr && pooled != nullptr && stats == nullptr && y2 == nullptr && H % 2 == 0 && W % 2 == 0)
               ? (u16*)pool : nullptr;
  a.ppitch = ppitch;
  // fused upsample needs the eval epilogue, 16-channel groups and the LDS band (<= 64 KB). Measured
  // (serving frame, N = 1): it wins only at the 16^2 bottleneck (6.9 us vs 4.8 + 4.8 us); at 32^2 /
  // 64^2 / 128^2 the banded two-phase kernel is slower than reduce + upsample (10.9 / 13.2 / 15.4 vs
  // 9.8 / 10.3 / 10.6 us; 2-row bands x 8 channels were slower still), so larger maps take the
  // separate upsample launch.
  const bool up_ok = up != nullptr && pooled != nullptr && pool == nullptr && stats == nullptr && y2 == nullptr &&
                     escale != nullptr && eshift != nullptr && Cout % UP_CG == 0 && upitch % 4 == 0 &&
                     (long)(UP_TY / 2 + 2) * W * UP_CG * 2 <= 65536 && uH >= 2 * H && uW >= 2 * W &&
                     (long)H * W <= 256;
  a.up = up_ok ? (u16*)up : nullptr;
  a.upitch = upitch; a.uH = uH; a.uW = uW; a.uoy = uoy; a.uox = uox;
  a.urh = 2 * H > 1 ? (float)(H - 1) / (float)(2 * H - 1) : 0.f;  // = ac_scale (pool_up.hip)
  a.urw = 2 * W > 1 ? (float)(W - 1) / (float)(2 * W - 1) : 0.f;
  long wse = has_ws ? ws_elems : 0;
  wse = wse < (1L << 29) ? wse : (1L << 29);  // slab bytes < 2 GiB (buffer offsets)
  a.x1 = (const u16*)x1; a.x2 = (const u16*)x2;
  a.xbytes1 = (uint32_t)xbytes1; a.xbytes2 = (uint32_t)xbytes2;
  a.C1 = C1; a.C2 = C2; a.pitch1 = pitch1; a.pitch2 = pitch2;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y1 = (u16*)y1; a.y2 = (u16*)y2; a.ybytes1 = (uint32_t)ybytes1; a.ybytes2 = (uint32_t)ybytes2;
  a.Cy1 = Cy1; a.ypitch1 = ypitch1; a.ypitch2 = ypitch2; a.stats = stats;
  if (bnpart && bny && bncoef && !stats && !escale && y2 == nullptr && Cy1 == Cout && bnypitch % 4 == 0 &&
      pool == nullptr && up == nullptr) {
    a.bny = (const u16*)bny; a.bnypitch = bnypitch; a.bncoef = bncoef; a.bnpart = bnpart; a.bnrows = bnrows;
  }
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
  if (Cout % 64 || Cy1 % 8) return -1;  // widened 16-B epilogue stores never straddle the split
  if (xbytes1 >= (1l << 31) || xbytes2 >= (1l << 31) || ybytes1 >= (1l << 31) || ybytes2 >= (1l << 31)) return -1;
  const FastDiv fhw = make_fastdiv((uint32_t)(H * W)), fw = make_fastdiv((uint32_t)W);
  a.fhw_m = fhw.m; a.fhw_s = fhw.s; a.fw_m = fw.m; a.fw_s = fw.s;
  // bm_pref: 0 = auto, 128 / 256 = force the tile; +1000*k: k = blocks per CU of the persistent
  // grid (k = 0 => 2 per CU, every block resident; large k ~ one tile per block)
  int per_cu = bm_pref / 1000;
  bm_pref %= 1000;
  if (per_cu == 0) per_cu = 2;  // default: 2 blocks per CU, every block resident
  // bm_pref 4 / 5: force the ping-pong 256 x 256 / 256 x 128 kernel (conv_pp_kernel)
  if (bm_pref == 4) return launch_pp<256>(a, s);
  if (bm_pref == 5) return launch_pp<128>(a, s);
  // auto: the ping-pong 256 x 256 kernel wherever its tile grid fills the chip (>= 256 tiles of 256
  // pixels x 256 couts; fewer tiles leave CUs idle at one block per CU). Measured
  // (scripts/conv_microbench.py, bs 64, one MI355X): 64^2 256->256 903 -> 1082 TF/s, 32^2 512->512
  // 962 -> 1205, 32^2 512+512->256 927 -> 1120; bs 64 step 2973 -> 3150 img/s. The 256 x 128 form is
  // 2-4 % faster than the 128 x 128 kernel where K >= 1152 (128^2 128->128 851 -> 889, 64^2
  // 256+256->128 882 -> 907; slower at K = 576) and +1.0-1.4 % on the bs 64 step.
  if (bm_pref == 0 && !packed) {
    const long tiles256 = (long)(a.M + 255) / 256 * (Cout / 256);
    if (Cout % 256 == 0 && Cy1 % 32 == 0 && tiles256 >= 256 && escale == nullptr) return launch_pp<256>(a, s);
    // 256 x 128 form: only where K is long enough (>= 128 input channels)
    const long tiles128 = (long)(a.M + 255) / 256 * (Cout / 128);
    if (Cout % 128 == 0 && Cy1 % 32 == 0 && tiles128 >= 256 && C1 + C2 >= 128 && escale == nullptr)
      return launch_pp<128>(a, s);
  }
  // bm_pref 7 / 8: force the split-K ping-pong 256 x 128 / 256 x 256 kernel (pp_split_plan's split)
  if (bm_pref == 7 || bm_pref == 8) {
    const int d = pp_split_plan(a.M, Cout, bm_pref == 7 ? 128 : 256, a.nks, wse);
    if (d < 2 || packed || Cy1 % 32) return -1;
    return bm_pref == 7 ? launch_pp<128>(a, s, d, pooled) : launch_pp<256>(a, s, d, pooled);
  }
  // auto, small M x long K (training): split-K ping-pong 256 x 128 where its plan exists and the 128 x 128
  // kernel would split K too (measured, scripts/conv_microbench.py --batch 4 --ws 1, one MI355X: 32^2
  // 1024->512 63.5 -> 53.2 us, 512->512 39.9 -> 36.7, 512+512->256 39.0 -> 36.7, 64^2 256->128 31.5 ->
  // 29.4; where the 128 x 128 grid needs no split (64^2 256->256) the unsplit kernel wins, 32.9 vs 39.5,
  // and at M = 1024 (16^2 512->1024: 29.5 vs 31.0 us) the 128 x 128 split does)
  // (eval too, BN fold in the shared reduce: the batched serving network at N = 4, scripts/rowband_bench.py
  // --batch 4 --variants 0,7: 32^2 1024->512 63.2 -> 52.3 us, 512->512 + pool 39.3 -> 36.4)
  if (bm_pref == 0 && !packed && Cout % 128 == 0 && Cy1 % 32 == 0 && C1 + C2 >= 128 &&
      a.M >= 4096 && (long)(a.M + 127) / 128 * (Cout / 128) < 192 && pp_split_enabled()) {
    const int d = pp_split_plan(a.M, Cout, 128, a.nks, wse);
    if (d > 1) return launch_pp<128>(a, s, d, pooled);
  }
  const int max_blocks = 256 * per_cu;
  // bm_pref 2 / 3: 8-wave blocks (64 x 32 per wave; twice the waves per SIMD to hide the per-step
  // barrier + DMA latency, 1.5x the LDS fragment reads per MFMA) for the 128x128 / 256x64 tiles
  // (measured dead end: 256 x 256 / 256 x 128 tiles in this 2-phase structure, one 8-wave block
  // per CU -- 49 spilled VGPRs at 256 x 256; +6 % on 32^2 x 512 -> 512 only, -5..-40 % elsewhere)
  if (bm_pref == 2 && Cout % 128 == 0) return launch_cfg<128, 128, 8>(a, max_blocks, wse, s, pooled);
  if (bm_pref == 3) return launch_cfg<256, 64, 8>(a, max_blocks, wse, s, pooled);
  if (bm_pref == 128 && Cout % 128 == 0) return launch_cfg<128, 128>(a, max_blocks, wse, s, pooled);
  if (bm_pref == 0 && Cout % 128 == 0) return launch_cfg<128, 128, 8>(a, max_blocks, wse, s, pooled);
  if (bm_pref == 256) return launch_cfg<256, 64>(a, max_blocks, wse, s, pooled);
  return launch_cfg<256, 64, 8>(a, max_blocks, wse, s, pooled);
}

// fp32 workspace elements the auto dispatch would use for split-K on this shape (0 = no split)
extern "C" long rdp_conv_ws_elems(int N, int H, int W, int C1, int C2, int Cout, int taps, int packed, int bm_pref) {
  const int pref = bm_pref % 1000;
  const int ht = rdp_conv_halo_tiles(N, H, W, C1, C2, Cout, taps, packed);
  if (ht > 0 && (pref == 1 || (pref == 0 && ht >= 256 && Cout == 64 && C1 + C2 >= 256))) return 0;
  if (packed) return 0;
  const int M = N * H * W;
  const int nks = taps * ((C1 + C2) / 64);
  const int BM = ((pref == 128 || pref == 0) && Cout % 128 == 0) ? 128 : 256, BN = BM == 128 ? 128 : 64;
  const int ntiles = (M + BM - 1) / BM * (Cout / BN);
  const int d = choose_ksplit(ntiles, nks, M, Cout, packed, 1L << 29);
  long need = d > 1 ? (long)d * M * Cout : 0;
  // the split-K ping-pong plan (auto at >= 128 input channels, or forced by bm_pref 7 / 8)
  if ((pref == 0 && C1 + C2 >= 128 && Cout % 128 == 0 && M >= 4096 && (long)(M + 127) / 128 * (Cout / 128) < 192) ||
      pref == 7 ||
      pref == 8) {
    const int dp = pp_split_plan(M, Cout, pref == 8 ? 256 : 128, nks, 1L << 29);
    if (dp > 1 && (long)dp * M * Cout > need) need = (long)dp * M * Cout;
  }
  return need;
}
