// Row-ring 3x3 convolution (stride 1, pad 1) for the 64-input-channel layers at W % 64 == 0: the
// forward of inc.double_conv.3 / up4.conv.double_conv.3 (64 -> 64) and down1...double_conv.0
// (64 -> 128), and the dgrad of inc.3 / up4.3 (64 -> 64) and of up4.conv.double_conv.0 (64 -> 64 + 64
// into the skip / upsample halves of the concat)
// (/root/reference/pkg/segmentation_model.py:34 DoubleConv conv2 at 256^2; autograd's
// conv backward for it, scripts/train_segmenter.py:162).
//
// Why a separate kernel: at 64 output channels the implicit-GEMM kernel (conv_igemm.hip) re-stages
// its 256-pixel A tile for every one of the 9 taps -- ~3 MFMAs per 1-KiB LDS-DMA piece -- and runs
// at the L2 -> LDS gather rate (~540-580 TF/s), not the MFMA rate. Here:
//   * the whole weight tensor (64 x 576 bf16 = 72 KiB) lives in VGPRs: every wave keeps the A
//     fragments of its 32 output channels for all 18 K-steps (144 VGPRs), loaded once per block;
//   * a block walks one 64-pixel column (image n, 64-pixel segment of the row) top to bottom, two
//     output rows per step; an output row needs input rows h-1, h, h+1, so a step stages only the
//     TWO new input rows (66 pixels x 128 B each, zero halo by out-of-range offsets) into an
//     8-slot LDS ring -- ~32 MFMAs per DMA piece, 10x fewer than the implicit GEMM;
//   * the 9 taps read the staged rows at shifted offsets (B fragments, ds_read_b128 of 16 rows),
//     two steps of DMA stay in flight across the per-step barrier (counted vmcnt, asm LDS-DMA).
// At a column's first / last row the dr = -1 / +1 taps read an all-zero slot instead (the ring slot
// holds another column's row there: the zero padding row of this one). Epilogue: bf16 store (permlane16-widened, 16 B
// per lane), optional training BN statistics (per-block partial rows) or eval BN fold + ReLU.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

struct RingArgs {
  const u16* x;
  uint32_t xbytes;
  int pitch;
  const u16* w;  // [64][ldw], k = tap * 64 + cin
  uint32_t wbytes;
  int ldw;
  u16* y;
  uint32_t ybytes;
  int ypitch;
  u16* y2;  // output channels >= Cy1 go here (dgrad of a concatenated input), or nullptr
  uint32_t ybytes2;
  int ypitch2, Cy1;
  float* stats;  // [gridDim.x * NPG][2][COUT] partial (sum, sumsq) or nullptr
  const float* escale;
  const float* eshift;
  int erelu;
  // dgrad epilogue fused with the next BN backward reduction (stats != nullptr): per channel
  // sum(g) and sum(g * xhat), g = relu'(bny * scale + shift) * out; bncoef = [mean|invstd|scale|shift]
  const u16* bny;
  int bnypitch;
  const float* bncoef;
  // serving head (HEAD variant): mask[m] = (sum_c a[m][c] * hw[c] + hb > hthr) for the eval output a
  // (BN folded + ReLU, bf16-rounded); the 64-channel output itself is not stored
  const float* hw;
  const float* hb;
  float hthr;
  uint8_t* hmask;
  // eval MaxPool2d(2) of the output (POOL variant): pool [N][H/2][W/2][64] with pixel pitch ppitch
  u16* pool;
  int ppitch;
  // BNIN: the input is the previous layer's pre-BN output; its BN + ReLU (scale, shift per input
  // channel) is applied to the staged rows in LDS
  const float* iscale;
  const float* ishift;
  // BNIN, optional: the formed activation of the rows this block owns is also stored here (pixel pitch
  // apitch), so the layer's weight gradient can run the plain ring kernel on it (nullptr: not stored)
  u16* aout;
  uint32_t abytes;
  int apitch;
  int H, W, WS;  // WS = W / 64 segments per image row
  int nrows;     // N * WS * H: input rows in column order (R = column * H + h)
  int npairs;    // nrows / 2: steps (two output rows each)
  int pairs_per_block;
  uint32_t fh_m, fh_s, fs_m, fs_s;  // fast division by H and by WS
};

RDP_DEV uint32_t rdiv(uint32_t n, uint32_t m, uint32_t s) { return (__umulhi(n, m) + n) >> s; }

// COUT = 64: 8 waves = 2 channel groups x 4 pixel groups (32 px); COUT = 128: 4 x 2 (64 px).
// BNR: dgrad epilogue fused with the owner layer's BN-backward reduction (a separate instantiation:
// its y registers would otherwise cost every other variant 12 VGPRs -- spills at COUT = 128)
// HEAD (COUT = 64, eval): the serving 1x1 head + threshold in the epilogue (SURVEY.md §7.3 "Conv1x1
// head fused into the epilogue of up4.conv2"). A pixel's 64 channels live in two waves (cg = 0, 1):
// each reduces its 32 over the lane groups, cg = 1 leaves its partial in LDS (double-buffered by step
// parity), and cg = 0 finishes the pixel after the next step's barrier (the last step after a final
// barrier) and stores the u8 mask.
// POOL (COUT = 64, eval): MaxPool2d(2) of the output in the epilogue. A step's two output rows are
// one row of 2x2 windows (rows 2P, 2P + 1 with H even): horizontal pairs are neighbouring lanes (DPP
// swap), vertical pairs are the orow = 0 / 1 waves of a pixel group, exchanged through LDS (step-parity
// double buffer) and finished by the orow = 0 waves after the next barrier.
// BNIN (training forward, COUT = 64): the input rows are the producer layer's pre-BN output y and
// a = relu(y * scale + shift), rounded to bf16 exactly as bn_relu_apply_kernel does, is formed in LDS
// once per staged element -- by the wave whose DMA staged it, right after its own vmcnt wait, so the
// step's existing barrier publishes it -- instead of a separate apply pass writing and re-reading a
// (padding chunks stay zero: the conv pads the post-ReLU activation). With aout, the interior chunks of
// the rows the block owns (2 P0 .. 2 (P0 + nks) - 1) are also stored there; every staged chunk issues
// its store (the others at an out-of-range offset) so the per-wave vmcnt counts below stay fixed.
template <int COUT, bool BNR = false, bool HEAD = false, bool POOL = false, bool BNIN = false>
__global__ __launch_bounds__(512, 2) void conv_ring_kernel(const RingArgs a) {
  constexpr int NCG = COUT / 32, NPG = 8 / NCG;  // waves per channel group / per pixel group
  constexpr int PXW = 128 / NPG, NI = PXW / 16;  // pixels per wave (one output row half or whole)
  constexpr int XREG = 72 * 128;  // one ring slot: pixels w0-1 .. w0+70 of one input row (66 used)
  constexpr int NX = 8;           // ring slots: 4 rows in use + 2 steps x 2 rows in flight
  constexpr int PIECES = 18;      // 1-KiB DMA pieces per step (2 rows x 9)
  constexpr int MINPW = PIECES / 8;
  constexpr int HPART = HEAD ? 2 * NPG * PXW * 4 : 0;  // head partials [parity][pixel group][pixel]
  // pool halves [parity][wave][i][pixel pair][lane group] x 16 B (4 packed bf16 pairs)
  constexpr int PPART = POOL ? 2 * 8 * NI * 8 * 4 * 16 : 0;
  __shared__ __attribute__((aligned(16))) char ring[(NX + 1) * XREG + 4 * COUT * 4 + HPART + PPART];  // + zero slot, BN fold / BN-bwd coefs
  float* const efold = (float*)(ring + (NX + 1) * XREG);  // eval BN fold [scale | shift] (LDS, not VGPRs)
  float* const hpart = (float*)(ring + (NX + 1) * XREG + 4 * COUT * 4);
  uint4* const ppart = (uint4*)(ring + (NX + 1) * XREG + 4 * COUT * 4 + HPART);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave / NPG;  // output channels 32 cg .. 32 cg + 31
  const int pg = wave % NPG;  // pixel group: output row of the pair and first pixel
  const int orow = pg / (NPG / 2), px0 = PXW * (pg % (NPG / 2));

  const int P0 = blockIdx.x * a.pairs_per_block;
  const int nks = min(a.npairs, P0 + a.pairs_per_block) - P0;
  if (nks <= 0) return;

  const auto rx = make_rsrc(a.x, a.xbytes);
  const auto rw = make_rsrc(a.w, a.wbytes);
  // this wave's 32 output channels all go to one destination (Cy1 % 32 == 0)
  const bool d2 = 32 * cg >= a.Cy1;
  const auto ry = d2 ? make_rsrc(a.y2, a.ybytes2) : make_rsrc(a.y, a.ybytes);
  const int ypitch = d2 ? a.ypitch2 : a.ypitch;
  const int cbase = d2 ? 32 * cg - a.Cy1 : 32 * cg;

  // ---- weights -> registers: wa[ks][j] = W[32 cg + 16 j + (lane & 15)][32 ks + 8 (lane >> 4) .. +7]
  bf16x8 wa[18][2];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 32 * cg + 16 * j + (lane & 15);
      const uint32_t off = (uint32_t)(n * a.ldw + 32 * ks + 8 * (lane >> 4)) * 2u;
      const uint4 v = bload16(rw, off);
      wa[ks][j] = __builtin_bit_cast(bf16x8, v);
    }
  // Consume every weight register here, so hipcc waits for these loads before the ring DMAs are
  // issued. Otherwise its waits for them stay inside the step loop (the loop-header state merges
  // "loads pending" from the preheader) and their trailing vmcnt(0..2) drain the ring DMAs that
  // must stay in flight across the step barrier.
#pragma unroll
  for (int ks = 0; ks < 18; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(wa[ks][j]));

  // ---- ring DMA: input row R (column order) into slot R % NX ----
  const int gch = (lane & 7) ^ (lane >> 3);  // global 16-B chunk (LDS row & 7 == lane >> 3)
  auto row_base = [&](int R, int& m0, int& w0) {  // first pixel of the row segment; -1: no such row
    if (R < 0 || R >= a.nrows) { m0 = -1; w0 = 0; return; }
    const uint32_t col = rdiv((uint32_t)R, a.fh_m, a.fh_s);
    const int h = R - (int)col * a.H;
    const uint32_t n = rdiv(col, a.fs_m, a.fs_s);
    const int ws = (int)col - (int)n * a.WS;
    w0 = ws * 64;
    m0 = ((int)n * a.H + h) * a.W + w0;
  };
  // pieces p = 0..17 of stage P (rows 2P + 1 and 2P + 2), wave w issues p = w, w + 8, w + 16
  auto issue = [&](int P) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int p = wave + 8 * t;
      if (p >= PIECES) continue;  // wave-uniform
      const int rr = p >= 9 ? 1 : 0, pj = p - 9 * rr;
      const int R = 2 * P + 1 + rr;
      int m0, w0;
      row_base(R, m0, w0);
      const int j = pj * 8 + (lane >> 3);
      const bool ok = (m0 >= 0) & (j < 66) & inb(w0 - 1 + j, a.W);
      const uint32_t off = ok ? (uint32_t)((m0 + j - 1) * a.pitch + gch * 8) * 2u : RDP_OOB;
      dma16_async(rx, (lds_void*)(ring + ((R + NX) % NX) * XREG + pj * 1024), off);
    }
  };
  auto issue_row = [&](int R) {  // prologue rows: 9 pieces of one row (wave 0 also takes piece 8)
    int m0, w0;
    row_base(R, m0, w0);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int pj = wave + 8 * t;
      if (pj >= 9) continue;  // wave-uniform
      const int j = pj * 8 + (lane >> 3);
      const bool ok = (m0 >= 0) & (j < 66) & inb(w0 - 1 + j, a.W);
      const uint32_t off = ok ? (uint32_t)((m0 + j - 1) * a.pitch + gch * 8) * 2u : RDP_OOB;
      dma16_async(rx, (lds_void*)(ring + ((R + NX) % NX) * XREG + pj * 1024), off);
    }
  };

  f32x4 acc[2][NI];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[2][4], s2[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
  if (a.escale) {
    for (int c = threadIdx.x; c < COUT; c += 512) { efold[c] = a.escale[c]; efold[COUT + c] = a.eshift[c]; }
  }
  if constexpr (BNR) {
    for (int c = threadIdx.x; c < 4 * COUT; c += 512) efold[c] = a.bncoef[c];
  }
  if constexpr (BNIN) {  // input BN [scale | shift] (64 input channels), visible before the first transform
    for (int c = threadIdx.x; c < 64; c += 512) { efold[c] = a.iscale[c]; efold[64 + c] = a.ishift[c]; }
    __syncthreads();
  }
  // BNIN: this lane's chunk of piece pj of input row R (staged by this wave): y -> relu(y*scale+shift)
  const auto ra = make_rsrc(a.aout, a.aout ? a.abytes : 0u);
  const int rown0 = 2 * P0, rown1 = 2 * (P0 + nks);  // rows this block owns (activation store)
  // cf = this lane's [scale x 8 | shift x 8] (its chunk's channels 8 gch ..), read once per stage
  auto bn_coefs = [&](float (&cf)[16]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { cf[k] = efold[8 * gch + k]; cf[8 + k] = efold[64 + 8 * gch + k]; }
  };
  auto bn_chunk = [&](int R, int pj, const float (&cf)[16]) {
    int m0, w0;
    row_base(R, m0, w0);
    const int j = pj * 8 + (lane >> 3);
    const bool ok = (m0 >= 0) & (j < 66) & inb(w0 - 1 + j, a.W);  // else padding: stays zero
    uint4* p = (uint4*)(ring + ((R + NX) % NX) * XREG + pj * 1024 + lane * 16);
    const uint4 v = *p;
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    const float* sc = cf;
    const float* sh = cf + 8;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = fmaxf(fmaf(__uint_as_float(wv[k] << 16), sc[2 * k], sh[2 * k]), 0.f);
      const float hi = fmaxf(fmaf(__uint_as_float(wv[k] & 0xffff0000u), sc[2 * k + 1], sh[2 * k + 1]), 0.f);
      o[k] = pack2bf(lo, hi);
    }
    const uint4 ov = make_uint4(o[0], o[1], o[2], o[3]);
    if (ok) *p = ov;
    const bool st = ok & (j >= 1) & (j <= 64) & (R >= rown0) & (R < rown1);
    bstore16(ra, st ? (uint32_t)((m0 + j - 1) * a.apitch + gch * 8) * 2u : RDP_OOB, ov);
  };
  auto bn_stage = [&](int P) {  // the pieces this wave staged for stage P (see issue)
    float cf[16];
    bn_coefs(cf);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int p = wave + 8 * t;
      if (p >= PIECES) continue;
      const int rr = p >= 9 ? 1 : 0;
      bn_chunk(2 * P + 1 + rr, p - 9 * rr, cf);
    }
  };
  auto bn_row = [&](int R) {  // the prologue pieces this wave staged for row R (see issue_row)
    float cf[16];
    bn_coefs(cf);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int pj = wave + 8 * t;
      if (pj < 9) bn_chunk(R, pj, cf);
    }
  };

  // slot NX stays zero: the padding row read by a column's first / last output row, so the tap loop
  // has no branches and the compiler can overlap one tap's fragment reads with the previous MFMAs
  for (int o = threadIdx.x * 16; o < XREG; o += 512 * 16) *(uint4*)(ring + NX * XREG + o) = make_uint4(0, 0, 0, 0);

  // prologue: rows 2 P0 - 1 (wave 0..8, one row) and 2 P0, then stages P0 and P0 + 1
  issue_row(2 * P0 - 1);
  issue_row(2 * P0);
  issue(P0);
  if (nks > 1) issue(P0 + 1);

  // fragment read geometry: B rows = pixels px0 + 16 i + (lane & 15) (+ ds + 1), chunk (lane >> 4)
  // (+ 4 for the second K-half of a tap), XOR-swizzled by the LDS row
  const int gq = lane >> 4;
  const int coff = 16 * (gq & 1) + 8 * (gq >> 1);  // this lane's 8 channels after the pair swap

  // head: this lane's 8 head weights (channels 32 cg + 16 j + 4 gq + r), the previous step's own
  // partials (cg = 0) and output row
  float hwl[2][4];
  float hprev[NI];
  int hm_prev = -1;
  if constexpr (HEAD) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) hwl[j][r] = a.hw[32 * cg + 16 * j + 4 * gq + r];
#pragma unroll
    for (int i = 0; i < NI; ++i) hprev[i] = 0.f;
  }
  const float hbias = HEAD ? a.hb[0] : 0.f;
  // pool: pooled-row base of the previous step's windows; orow = 0 waves finish them
  int pb_prev = -1;
  auto pool_finish = [&](int par) {
    if (orow != 0 || pb_prev < 0) return;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (lane & 1) continue;
      const int q = (lane & 15) >> 1;
      const uint4 u0 = ppart[(((par * 8 + wave) * NI + i) * 8 + q) * 4 + gq];
      const uint4 u1 = ppart[(((par * 8 + wave + NPG / 2) * NI + i) * 8 + q) * 4 + gq];
      const uint32_t w0[4] = {u0.x, u0.y, u0.z, u0.w}, w1[4] = {u1.x, u1.y, u1.z, u1.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(__uint_as_float(w0[k] << 16), __uint_as_float(w1[k] << 16));
        const float hi = fmaxf(__uint_as_float(w0[k] & 0xffff0000u), __uint_as_float(w1[k] & 0xffff0000u));
        o[k] = pack2bf(lo, hi);
      }
      u16* dst = a.pool + (size_t)(pb_prev + ((px0 + 16 * i + (lane & 15)) >> 1)) * a.ppitch + 32 * cg + 4 * gq;
      *(uint2*)dst = make_uint2(o[0], o[1]);         // channels 32 cg + 4 gq .. + 3
      *(uint2*)(dst + 16) = make_uint2(o[2], o[3]);  // channels 32 cg + 16 + 4 gq .. + 3
    }
  };
  // cg = 0: finish the pixels of the step whose partials (parity par) are in LDS
  auto head_finish = [&](int par) {
    if (cg != 0 || hm_prev < 0) return;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int px = 16 * i + (lane & 15);
      const float x = hprev[i] + hpart[(par * NPG + pg) * PXW + px] + hbias;
      if (lane < 16) a.hmask[hm_prev + px0 + px] = x > a.hthr ? 1 : 0;
    }
  };

  for (int ks = 0; ks < nks; ++ks) {
    const int P = P0 + ks;
    // Stage P must have landed. vmcnt also counts the NI output stores every wave issues at the end
    // of a step, in issue order: younger than stage P are the stores of steps ks-2 and ks-1 and
    // (unless this is the last step) stage P+1 -- leave exactly those in flight.
    // (HEAD: no activation stores; the mask stores of cg = 0 are not counted, which only makes the
    // wait stricter)
    // BNIN: also the activation stores of step ks - 1's transform, younger than stage P's DMAs: at
    // least AS per wave per stage (2 or 3 pieces) and AS0 at step 0 (+ the 1-2 pieces of each prologue row)
    constexpr int NS = HEAD ? 0 : NI;  // counted output stores per step
    constexpr int AS = BNIN ? 2 : 0, AS0 = BNIN ? 4 : 0;
    if (ks + 1 < nks) {
      if (ks >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(MINPW + 2 * NS + AS) : "memory");
      else if (ks == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(MINPW + NS + AS0) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(MINPW) : "memory");
    } else {
      if (ks >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NS + AS) : "memory");
      else if (ks == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NS + AS0) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    if constexpr (BNIN) {  // this wave's DMAs of stage P (and at the start the prologue rows) have landed
      if (ks == 0) {
        bn_row(2 * P0 - 1);
        bn_row(2 * P0);
      }
      bn_stage(P);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    raw_barrier();
    if constexpr (HEAD) head_finish((ks - 1) & 1);
    if constexpr (POOL) pool_finish((ks - 1) & 1);
    // BN-backward fusion: the owner layer's pre-BN activations at this step's outputs, loaded before
    // the stage P + 2 DMAs so their latency hides under the taps. (hipcc cannot see the DMAs, so its
    // vmcnt(0) before the first use also waits for stage P + 2; keeping the loads invisible to it with
    // inline asm + a hand-counted vmcnt is unsafe: it may copy the destination registers before the wait.)
    uint2 yb[NI][2];
    if constexpr (BNR) {
      int ym0, yw0;
      row_base(2 * P + orow, ym0, yw0);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const u16* pa = a.bny + (size_t)(ym0 + px0 + 16 * i + (lane & 15)) * a.bnypitch + 32 * cg + 16 * j + 4 * gq;
          yb[i][j] = *(const uint2*)pa;
        }
    }
    const bool dma_next = ks + 2 < nks;
    if (dma_next) issue(P + 2);

    const int R0 = 2 * P + orow;  // this wave's output row (column order)
    const int h = R0 - (int)rdiv((uint32_t)R0, a.fh_m, a.fh_s) * a.H;
    const bool top = h == 0, bottom = h == a.H - 1;
    // software-pipelined over the 9 taps: the 4 B fragments of tap t + 1 are read while tap t's 8
    // MFMAs run (with only 2 waves per SIMD, a read -> wait -> MFMA chain per tap leaves the
    // matrix pipe idle for the LDS latency)
    auto tap_base = [&](int tap) {
      const int dr = tap / 3 - 1;
      const bool pad = (dr < 0 && top) || (dr > 0 && bottom);  // wave-uniform
      return ring + (pad ? NX : (R0 + dr + NX) % NX) * XREG;
    };
    auto read_tap = [&](int tap, bf16x8 (&fb)[2][NI]) {
      const char* xb = tap_base(tap);
      const int ds = tap % 3 - 1;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int row = px0 + 16 * i + (lane & 15) + ds + 1;
          fb[kh][i] = *(const bf16x8*)(xb + row * 128 + 16 * ((gq + 4 * kh) ^ (row & 7)));
        }
    };
    // (NI = 4 has twice the MFMAs per fragment read and no registers for a second set: no pipelining)
    constexpr bool PIPE = NI <= 2;
    if constexpr (!PIPE) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const char* xb = tap_base(tap);
        const int ds = tap % 3 - 1;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          bf16x8 fb[NI];
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const int row = px0 + 16 * i + (lane & 15) + ds + 1;
            fb[i] = *(const bf16x8*)(xb + row * 128 + 16 * ((gq + 4 * kh) ^ (row & 7)));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < NI; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[2 * tap + kh][j], fb[i], acc[j][i], 0, 0, 0);
        }
      }
    }
    bf16x8 fcur[2][NI], fnxt[2][NI];
    if (PIPE) read_tap(0, fcur);
#pragma unroll
    for (int tap = 0; tap < 9 && PIPE; ++tap) {
      if (PIPE && tap + 1 < 9) read_tap(tap + 1, fnxt);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < NI; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[2 * tap + kh][j], fcur[kh][i], acc[j][i], 0, 0, 0);
      if (PIPE && tap + 1 < 9) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < NI; ++i) fcur[kh][i] = fnxt[kh][i];
      }
    }

    // ---- epilogue of the step: acc[j][i][r] = out[pixel px0 + 16 i + (lane & 15)][cout 32 cg + 16 j + 4 gq + r]
    int m0, w0;
    row_base(R0, m0, w0);
    if constexpr (POOL) pb_prev = (((m0 - w0) / a.W) >> 1) * (a.W >> 1) + (w0 >> 1);
    if constexpr (HEAD) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float p = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 o = acc[j][i];
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int c = 32 * cg + 16 * j + 4 * gq;
          const float4 sc = *(const float4*)(efold + c), sh = *(const float4*)(efold + COUT + c);
          o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
          o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float q = bf2f(f2bf(fmaxf(o[r], 0.f)));  // the bf16 activation the unfused head reads
            p = fmaf(q, hwl[j][r], p);
          }
        }
        p += __shfl_xor(p, 16, 64);
        p += __shfl_xor(p, 32, 64);
        if (cg == 1) {
          if (lane < 16) hpart[((ks & 1) * NPG + pg) * PXW + 16 * i + lane] = p;
        } else {
          hprev[i] = p;
        }
      }
      hm_prev = m0;
      continue;  // no activation output in head mode
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint2 v[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 o = acc[j][i];
        acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (a.escale) {
          const int c = 32 * cg + 16 * j + 4 * gq;
          const float4 sc = *(const float4*)(efold + c), sh = *(const float4*)(efold + COUT + c);
          o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
          o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
          if (a.erelu) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
          }
        }
        v[j].x = pack2bf(o[0], o[1]);
        v[j].y = pack2bf(o[2], o[3]);
        if (a.stats) {
          const float q0 = __uint_as_float(v[j].x << 16), q1 = __uint_as_float(v[j].x & 0xffff0000u);
          const float q2 = __uint_as_float(v[j].y << 16), q3 = __uint_as_float(v[j].y & 0xffff0000u);
          if constexpr (BNR) {
            const int c = 32 * cg + 16 * j + 4 * gq;
            const float4 mu = *(const float4*)(efold + c), iv = *(const float4*)(efold + COUT + c);
            const float4 sc = *(const float4*)(efold + 2 * COUT + c), sh = *(const float4*)(efold + 3 * COUT + c);
            const float y0 = __uint_as_float(yb[i][j].x << 16), y1 = __uint_as_float(yb[i][j].x & 0xffff0000u);
            const float y2 = __uint_as_float(yb[i][j].y << 16), y3 = __uint_as_float(yb[i][j].y & 0xffff0000u);
            const float g0 = fmaf(y0, sc.x, sh.x) > 0.f ? q0 : 0.f, g1 = fmaf(y1, sc.y, sh.y) > 0.f ? q1 : 0.f;
            const float g2 = fmaf(y2, sc.z, sh.z) > 0.f ? q2 : 0.f, g3 = fmaf(y3, sc.w, sh.w) > 0.f ? q3 : 0.f;
            s1[j][0] += g0; s2[j][0] += g0 * (y0 - mu.x) * iv.x;
            s1[j][1] += g1; s2[j][1] += g1 * (y1 - mu.y) * iv.y;
            s1[j][2] += g2; s2[j][2] += g2 * (y2 - mu.z) * iv.z;
            s1[j][3] += g3; s2[j][3] += g3 * (y3 - mu.w) * iv.w;
          } else {
            s1[j][0] += q0; s2[j][0] += q0 * q0;
            s1[j][1] += q1; s2[j][1] += q1 * q1;
            s1[j][2] += q2; s2[j][2] += q2 * q2;
            s1[j][3] += q3; s2[j][3] += q3 * q3;
          }
        }
      }
      if constexpr (POOL) {  // horizontal max with the neighbouring pixel (lane ^ 1), half to LDS
        uint32_t hw4[4] = {v[0].x, v[0].y, v[1].x, v[1].y};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hw4[k], 0xB1, 0xf, 0xf, false);
          const float lo = fmaxf(__uint_as_float(hw4[k] << 16), __uint_as_float(nb << 16));
          const float hi = fmaxf(__uint_as_float(hw4[k] & 0xffff0000u), __uint_as_float(nb & 0xffff0000u));
          hw4[k] = pack2bf(lo, hi);
        }
        if (!(lane & 1))
          ppart[((((ks & 1) * 8 + wave) * NI + i) * 8 + ((lane & 15) >> 1)) * 4 + gq] =
              make_uint4(hw4[0], hw4[1], hw4[2], hw4[3]);
      }
      const auto rxs = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
      const auto rys = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
      const int m = m0 + px0 + 16 * i + (lane & 15);
      const uint32_t off = (uint32_t)(m * ypitch + cbase + coff) * 2u;
      bstore16(ry, off, make_uint4(rxs[0], rys[0], rxs[1], rys[1]));
    }
  }

  if constexpr (HEAD) {
    __syncthreads();
    head_finish((nks - 1) & 1);
    return;
  }
  if constexpr (POOL) {
    __syncthreads();
    pool_finish((nks - 1) & 1);
  }
  if (a.stats) {  // one partial row per (block, pixel group); waves cg = 0 / 1 fill its two halves
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] = row16_sum(s1[j][r]);
        s2[j][r] = row16_sum(s2[j][r]);
      }
    if ((lane & 15) == 0) {
      float* row = a.stats + (size_t)(blockIdx.x * NPG + pg) * 2 * COUT;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 32 * cg + 16 * j + 4 * gq;
        *(float4*)(row + c) = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
        *(float4*)(row + COUT + c) = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
      }
    }
  }
}

// Applicability of the ring kernel (3x3, one 64-channel source, 64 or 128 outputs -- split at a
// multiple of 32 into two destinations --, W % 64 == 0, even H); returns the stats rows it writes,
// or -1 when not applicable.
extern "C" int rdp_conv_ring_ex(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                                void* y, long ybytes, int ypitch, void* y2, long ybytes2, int ypitch2, int Cy1,
                                int Cout, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                                int erelu, int max_blocks, const void* bn_y_, int bn_ypitch, const float* bn_coef,
                                const float* iscale, const float* ishift, void* aout, long abytes, int apitch,
                                hipStream_t s);
extern "C" int rdp_conv_ring(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                             void* y, long ybytes, int ypitch, void* y2, long ybytes2, int ypitch2, int Cy1,
                             int Cout, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                             int erelu, int max_blocks, hipStream_t s) {
  return rdp_conv_ring_ex(x, xbytes, C, pitch, w, wbytes, ldw, y, ybytes, ypitch, y2, ybytes2, ypitch2, Cy1, Cout,
                          stats, N, H, W, escale, eshift, erelu, max_blocks, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                          0, 0, s);
}

// Eval conv (64 -> 64, BN folded + ReLU) fused with the serving 1x1 head: writes only the u8 mask
// (logit > thr) of the 64-channel output. Returns 0, or -1 when the ring kernel does not apply.
extern "C" int rdp_conv_ring_head(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                                  int Cout, int N, int H, int W, const float* escale, const float* eshift,
                                  const float* hw, const float* hb, float hthr, void* mask, hipStream_t s) {
  if (C != 64 || Cout != 64 || W % 64 || H % 2 || ldw < 576 || !escale || !eshift || !hw || !hb || !mask) return -1;
  if (xbytes >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  RingArgs a;
  a.x = (const u16*)x; a.xbytes = (uint32_t)xbytes; a.pitch = pitch;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y = nullptr; a.ybytes = 0; a.ypitch = 64; a.y2 = nullptr; a.ybytes2 = 0; a.ypitch2 = 64; a.Cy1 = 64;
  a.stats = nullptr; a.escale = escale; a.eshift = eshift; a.erelu = 1;
  a.bny = nullptr; a.bnypitch = 0; a.bncoef = nullptr;
  a.hw = hw; a.hb = hb; a.hthr = hthr; a.hmask = (uint8_t*)mask;
  a.pool = nullptr; a.ppitch = 0;
  a.iscale = nullptr; a.ishift = nullptr;
  a.aout = nullptr; a.abytes = 0; a.apitch = 0;
  a.H = H; a.W = W; a.WS = W / 64;
  a.nrows = N * a.WS * H;
  a.npairs = a.nrows / 2;
  const int blocks = std::max(1, std::min(256, a.npairs));
  a.pairs_per_block = (a.npairs + blocks - 1) / blocks;
  const int grid = (a.npairs + a.pairs_per_block - 1) / a.pairs_per_block;
  const FastDiv fh = make_fastdiv((uint32_t)H), fs = make_fastdiv((uint32_t)a.WS);
  a.fh_m = fh.m; a.fh_s = fh.s; a.fs_m = fs.m; a.fs_s = fs.s;
  hipLaunchKernelGGL((conv_ring_kernel<64, false, true>), dim3(grid), dim3(512), 0, s, a);
  return 0;
}

// Eval conv (64 -> 64, BN folded + ReLU) that also writes MaxPool2d(2) of its output into pool
// [N][H/2][W/2][64] (pixel pitch ppitch). Returns 0, or -1 when the ring kernel does not apply.
extern "C" int rdp_conv_ring_pool(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                                  void* y, long ybytes, int ypitch, int Cout, int N, int H, int W,
                                  const float* escale, const float* eshift, int erelu, void* pool, int ppitch,
                                  hipStream_t s) {
  if (C != 64 || Cout != 64 || W % 64 || H % 2 || ldw < 576 || !escale || !eshift || !pool || ppitch % 4) return -1;
  if (xbytes >= (1l << 31) || ybytes >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  RingArgs a;
  a.x = (const u16*)x; a.xbytes = (uint32_t)xbytes; a.pitch = pitch;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.y2 = (u16*)y; a.ybytes2 = 0; a.ypitch2 = ypitch; a.Cy1 = 64;
  a.stats = nullptr; a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  a.bny = nullptr; a.bnypitch = 0; a.bncoef = nullptr;
  a.hw = nullptr; a.hb = nullptr; a.hthr = 0.f; a.hmask = nullptr;
  a.pool = (u16*)pool; a.ppitch = ppitch;
  a.iscale = nullptr; a.ishift = nullptr;
  a.aout = nullptr; a.abytes = 0; a.apitch = 0;
  a.H = H; a.W = W; a.WS = W / 64;
  a.nrows = N * a.WS * H;
  a.npairs = a.nrows / 2;
  const int blocks = std::max(1, std::min(256, a.npairs));
  a.pairs_per_block = (a.npairs + blocks - 1) / blocks;
  const int grid = (a.npairs + a.pairs_per_block - 1) / a.pairs_per_block;
  const FastDiv fh = make_fastdiv((uint32_t)H), fs = make_fastdiv((uint32_t)a.WS);
  a.fh_m = fh.m; a.fh_s = fh.s; a.fs_m = fs.m; a.fs_s = fs.s;
  hipLaunchKernelGGL((conv_ring_kernel<64, false, false, true>), dim3(grid), dim3(512), 0, s, a);
  return 0;
}

// Row-ring dgrad whose epilogue also produces the BN-backward partial rows of the layer that owns
// the output (bn_y: its pre-BN activations, bn_coef: its [mean|invstd|scale|shift]; ReLU applied):
// replaces a separate bn_relu_bwd_reduce pass over (da, y). Returns the partial rows, or -1.
extern "C" int rdp_conv_ring_ex(const void* x, long xbytes, int C, int pitch, const void* w, long wbytes, int ldw,
                                void* y, long ybytes, int ypitch, void* y2, long ybytes2, int ypitch2, int Cy1,
                                int Cout, float* stats, int N, int H, int W, const float* escale, const float* eshift,
                                int erelu, int max_blocks, const void* bn_y_, int bn_ypitch, const float* bn_coef,
                                const float* iscale, const float* ishift, void* aout, long abytes, int apitch,
                                hipStream_t s) {
  const u16* bn_y = (const u16*)bn_y_;
  if (aout && (!iscale || abytes >= (1l << 31) || apitch % 8)) return -1;
  if (bn_y && (!stats || escale || y2 || bn_ypitch % 4 || Cout != 64)) return -1;
  if (iscale && (!ishift || bn_y || escale || y2 || Cout != 64)) return -1;
  if (C != 64 || (Cout != 64 && Cout != 128) || W % 64 || H % 2 || ldw < 576 || Cy1 % 32) return -1;
  if (y2 == nullptr && Cy1 != Cout) return -1;
  if (xbytes >= (1l << 31) || ybytes >= (1l << 31) || ybytes2 >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  RingArgs a;
  a.x = (const u16*)x; a.xbytes = (uint32_t)xbytes; a.pitch = pitch;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.y2 = (u16*)(y2 ? y2 : y); a.ybytes2 = y2 ? (uint32_t)ybytes2 : 0u; a.ypitch2 = y2 ? ypitch2 : ypitch;
  a.Cy1 = Cy1;
  a.stats = stats; a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  a.bny = bn_y; a.bnypitch = bn_ypitch; a.bncoef = bn_coef;
  a.hw = nullptr; a.hb = nullptr; a.hthr = 0.f; a.hmask = nullptr;
  a.pool = nullptr; a.ppitch = 0;
  a.iscale = iscale; a.ishift = ishift;
  a.aout = (u16*)aout; a.abytes = (uint32_t)abytes; a.apitch = apitch;
  a.H = H; a.W = W; a.WS = W / 64;
  a.nrows = N * a.WS * H;
  a.npairs = a.nrows / 2;
  const int blocks = std::max(1, std::min(max_blocks > 0 ? max_blocks : 256, a.npairs));
  a.pairs_per_block = (a.npairs + blocks - 1) / blocks;
  const int grid = (a.npairs + a.pairs_per_block - 1) / a.pairs_per_block;
  const FastDiv fh = make_fastdiv((uint32_t)H), fs = make_fastdiv((uint32_t)a.WS);
  a.fh_m = fh.m; a.fh_s = fh.s; a.fs_m = fs.m; a.fs_s = fs.s;
  if (Cout == 128) {
    hipLaunchKernelGGL((conv_ring_kernel<128>), dim3(grid), dim3(512), 0, s, a);
    return grid * 2;
  }
  if (bn_y) {
    hipLaunchKernelGGL((conv_ring_kernel<64, true>), dim3(grid), dim3(512), 0, s, a);
    return grid * 4;
  }
  if (iscale) {
    hipLaunchKernelGGL((conv_ring_kernel<64, false, false, false, true>), dim3(grid), dim3(512), 0, s, a);
    return grid * 4;
  }
  hipLaunchKernelGGL((conv_ring_kernel<64>), dim3(grid), dim3(512), 0, s, a);
  return grid * 4;
}

// ---- two-source (128 -> 64) row ring ---------------------------------------------------------------
// The first conv of up4 (/root/reference/pkg/segmentation_model.py:62,75-76: DoubleConv(128, 64) on
// cat([skip, up]) at 256^2) and the second conv of up3 (128 -> 64 at 128^2) as a row ring: the 9 taps of
// 128 input channels, 64 outputs. The whole weight tensor (64 x 1152 bf16) does not fit one wave's
// registers, so K is split over wave pairs: 8 waves = 2 channel groups (32 outputs) x 2 K-halves (the
// 64 channels of source 0 / source 1: the skip and the upsample, or the two halves of one 128-channel
// tensor) x 2 output rows of the step; every wave keeps its 32 x 576 weights in VGPRs (144) and
// computes all 64 pixels of its row over its K-half. The two partial tiles of a (channel group, row)
// meet in LDS: each wave hands its partner the fp32 half of the tile the partner finishes (32 pixels),
// one barrier later adds the partner's half of its own, and runs the epilogue (bf16 store, BN
// statistics or eval BN fold + ReLU) on its 32 pixels. A ring slot holds one input row of both
// sources (2 x 72 x 128 B); 6 slots = the 4 rows of a step + the next stage's 2 rows in flight, so
// the ring + exchange tile + zero row fit the 160 KiB LDS with one 512-thread block per CU.
struct Ring2Args {
  const u16* x0;
  const u16* x1;
  uint32_t xbytes0, xbytes1;
  int pitch0, pitch1;
  const u16* w;  // [64][ldw], k = tap * 128 + 64 * source + cin
  uint32_t wbytes;
  int ldw;
  u16* y;
  uint32_t ybytes;
  int ypitch;
  float* stats;  // [gridDim.x * 4][2][scout] partial (sum, sumsq) at channels co0 .. co0 + 63, or nullptr
  int scout, co0;
  const float* escale;
  const float* eshift;
  int erelu;
  int H, W, WS, nrows, npairs, pairs_per_block;
  uint32_t fh_m, fh_s, fs_m, fs_s;
};

__global__ __launch_bounds__(512, 2) void conv_ring2_kernel(const Ring2Args a) {
  constexpr int XREG = 72 * 128;          // one source of one staged row
  constexpr int SLOT = 2 * XREG;          // both sources
  constexpr int NX = 6;                   // 4 rows in use + the next stage's 2
  constexpr int PIECES = 36;              // 1-KiB DMA pieces per stage: 2 rows x 2 sources x 9
  constexpr int MINPW = PIECES / 8;       // pieces of the wave that issues fewest
  constexpr int XCH = 2 * 2 * 2 * 2 * 2 * 64 * 16;  // exchange: [orow][cg][dst half][i2][j] x 64 lanes x 16 B
  __shared__ __attribute__((aligned(16))) char ring[NX * SLOT + XREG + XCH + 2 * 64 * 4];
  char* const zslot = ring + NX * SLOT;
  f32x4* const xch = (f32x4*)(ring + NX * SLOT + XREG);
  float* const efold = (float*)(ring + NX * SLOT + XREG + XCH);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave & 1, kh = (wave >> 1) & 1, orow = wave >> 2;

  const int P0 = blockIdx.x * a.pairs_per_block;
  const int nks = min(a.npairs, P0 + a.pairs_per_block) - P0;
  if (nks <= 0) return;

  const auto rx0 = make_rsrc(a.x0, a.xbytes0);
  const auto rx1 = make_rsrc(a.x1, a.xbytes1);
  const auto rw = make_rsrc(a.w, a.wbytes);
  const auto ry = make_rsrc(a.y, a.ybytes);

  // weights: wa[ks][j] = W[32 cg + 16 j + (lane & 15)][tap * 128 + 64 kh + 32 (ks & 1) + 8 (lane >> 4) .. +7]
  bf16x8 wa[18][2];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 32 * cg + 16 * j + (lane & 15);
      const uint32_t off = (uint32_t)(n * a.ldw + (ks >> 1) * 128 + 64 * kh + 32 * (ks & 1) + 8 * (lane >> 4)) * 2u;
      wa[ks][j] = __builtin_bit_cast(bf16x8, bload16(rw, off));
    }
#pragma unroll
  for (int ks = 0; ks < 18; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(wa[ks][j]));  // loads waited here, not in the loop

  // DMA lane geometry: LDS row pj * 8 + lrow, global 16-B chunk gch of it; per source the lane part
  // of the global offset (elements): lrow * pitch + 8 gch (the pieces add scalar parts only)
  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;
  const int lofs0 = lrow * a.pitch0 + gch * 8, lofs1 = lrow * a.pitch1 + gch * 8;
  auto row_base = [&](int R, int& m0, int& w0) {
    if (R < 0 || R >= a.nrows) { m0 = -1; w0 = 0; return; }
    const uint32_t col = rdiv((uint32_t)R, a.fh_m, a.fh_s);
    const int h = R - (int)col * a.H;
    const uint32_t n = rdiv(col, a.fs_m, a.fs_s);
    const int ws = (int)col - (int)n * a.WS;
    w0 = ws * 64;
    m0 = ((int)n * a.H + h) * a.W + w0;
  };
  // piece q (0..17) of row R: source q / 9, LDS row group q % 9
  auto dma_piece = [&](int R, int q, int lr) {
    int m0, w0;
    row_base(R, m0, w0);
    const int src = q >= 9 ? 1 : 0, pj = q - 9 * src;  // wave-uniform
    const int j = pj * 8 + lr;
    const bool ok = (m0 >= 0) & (j < 66) & inb(w0 - 1 + j, a.W);
    const int pitch = src ? a.pitch1 : a.pitch0;
    const uint32_t off = ok ? (uint32_t)((m0 + pj * 8 - 1) * pitch + (src ? lofs1 : lofs0)) * 2u : RDP_OOB;
    dma16_async(src ? rx1 : rx0, (lds_void*)(ring + ((R + NX) % NX) * SLOT + src * XREG + pj * 1024), off);
  };
  // (lr re-derived per call behind an opaque asm: per-piece lane values are recomputed, not hoisted
  // out of the step loop into registers the weights need)
  auto issue = [&](int P) {  // stage P = rows 2P + 1, 2P + 2: wave w issues pieces w, w + 8, ...
    int lr = lrow;
    asm volatile("" : "+v"(lr));
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int p = wave + 8 * t;
      if (p >= PIECES) continue;
      const int rr = p >= 18 ? 1 : 0;
      dma_piece(2 * P + 1 + rr, p - 18 * rr, lr);
    }
  };
  auto issue_row = [&](int R) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int q = wave + 8 * t;
      if (q < 18) dma_piece(R, q, lrow);
    }
  };

  for (int o = threadIdx.x * 16; o < XREG; o += 512 * 16) *(uint4*)(zslot + o) = make_uint4(0, 0, 0, 0);
  if (a.escale) {
    for (int c = threadIdx.x; c < 64; c += 512) { efold[c] = a.escale[c]; efold[64 + c] = a.eshift[c]; }
  }

  issue_row(2 * P0 - 1);
  issue_row(2 * P0);
  issue(P0);

  const int gq = lane >> 4;
  const int coff = 16 * (gq & 1) + 8 * (gq >> 1);
  int lpart[3][2];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int r = (lane & 15) + d;
      lpart[d][h2] = r * 128 + 16 * ((gq + 4 * h2) ^ (r & 7));
    }
  f32x4 acc[2][4];
  float s1[2][4], s2[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
  constexpr int NS = 2;  // output stores per wave per step (its 2 fragments of 16 pixels)

  for (int ks = 0; ks < nks; ++ks) {
    const int P = P0 + ks;
    // stage P landed; younger than it: only the NS stores of step ks - 1
    if (ks == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NS) : "memory");
    raw_barrier();  // every wave's stage P visible; every wave done with step ks - 1 (ring rows, exchange)
    asm volatile("" ::: "memory");  // no LDS access of this step moves above the barrier
    if (ks + 1 < nks) issue(P + 1);

    const int R0 = 2 * P + orow;
    const int h = R0 - (int)rdiv((uint32_t)R0, a.fh_m, a.fh_s) * a.H;
    const bool top = h == 0, bottom = h == a.H - 1;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto src_base = [&](int tap) {
      const int dr = tap / 3 - 1;
      const bool pad = (dr < 0 && top) || (dr > 0 && bottom);  // wave-uniform
      return pad ? zslot : ring + ((R0 + dr + NX) % NX) * SLOT + kh * XREG;
    };
    // fragment i of K-step kk: LDS row 16 i + (lane & 15) + ds + 1 of the tap's slot; the swizzle only
    // sees the row's low 3 bits, so the lane part is one of 6 offsets and 16 i a 2-KiB immediate
    auto read_frag = [&](int kk, bf16x8 (&fb)[4]) {  // kk = 2 tap + K-half of the source's 64 channels
      const char* xb = src_base(kk >> 1) + lpart[(kk >> 1) % 3][kk & 1];
#pragma unroll
      for (int i = 0; i < 4; ++i) fb[i] = *(const bf16x8*)(xb + 2048 * i);
    };
    // 18 K-steps of 4 fragment reads + 8 MFMAs (no second fragment set: the registers hold the weights;
    // the SIMD's other wave covers the read latency)
#pragma unroll
    for (int kk = 0; kk < 18; ++kk) {
      bf16x8 fb[4];
      read_frag(kk, fb);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[kk][j], fb[i], acc[j][i], 0, 0, 0);
    }

    // exchange: this wave finishes pixels 32 kh .. 32 kh + 31 (fragments 2 kh, 2 kh + 1); the partner
    // (same cg / row, other K-half) finishes the rest. kh is wave-uniform: scalar branches pick the
    // register sets (no dynamic register indexing, no second copy of the tile)
    const int xo = (orow * 2 + cg) * 2;  // [orow][cg] base, then [dst half][i2][j]
    auto give = [&](int ib) {  // fragments ib, ib + 1 -> the partner's slots
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int j = 0; j < 2; ++j) xch[(((xo + (1 - kh)) * 2 + i2) * 2 + j) * 64 + lane] = acc[j][ib + i2];
    };
    if (kh == 0) give(2);
    else give(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    asm volatile("" ::: "memory");

    int m0, w0;
    row_base(R0, m0, w0);
    auto finish = [&](int ib) {  // fragments ib, ib + 1 (+ the partner's partials) -> epilogue
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        const int i = ib + i2;
        uint2 v[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 o = acc[j][i] + xch[(((xo + kh) * 2 + i2) * 2 + j) * 64 + lane];
          if (a.escale) {
            const int c = 32 * cg + 16 * j + 4 * gq;
            const float4 sc = *(const float4*)(efold + c), sh = *(const float4*)(efold + 64 + c);
            o[0] = fmaf(o[0], sc.x, sh.x); o[1] = fmaf(o[1], sc.y, sh.y);
            o[2] = fmaf(o[2], sc.z, sh.z); o[3] = fmaf(o[3], sc.w, sh.w);
            if (a.erelu) {
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
            }
          }
          v[j].x = pack2bf(o[0], o[1]);
          v[j].y = pack2bf(o[2], o[3]);
          if (a.stats) {
            const float q0 = __uint_as_float(v[j].x << 16), q1 = __uint_as_float(v[j].x & 0xffff0000u);
            const float q2 = __uint_as_float(v[j].y << 16), q3 = __uint_as_float(v[j].y & 0xffff0000u);
            s1[j][0] += q0; s2[j][0] += q0 * q0;
            s1[j][1] += q1; s2[j][1] += q1 * q1;
            s1[j][2] += q2; s2[j][2] += q2 * q2;
            s1[j][3] += q3; s2[j][3] += q3 * q3;
          }
        }
        const auto rxs = __builtin_amdgcn_permlane16_swap(v[0].x, v[1].x, false, false);
        const auto rys = __builtin_amdgcn_permlane16_swap(v[0].y, v[1].y, false, false);
        const int m = m0 + 16 * i + (lane & 15);
        bstore16(ry, (uint32_t)(m * a.ypitch + 32 * cg + coff) * 2u, make_uint4(rxs[0], rys[0], rxs[1], rys[1]));
      }
    };
    if (kh == 0) finish(0);
    else finish(2);
  }

  if (a.stats) {  // one partial row per (block, row of the step, pixel half); cg = 0 / 1 fill its halves
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] = row16_sum(s1[j][r]);
        s2[j][r] = row16_sum(s2[j][r]);
      }
    if ((lane & 15) == 0) {
      float* row = a.stats + (size_t)(blockIdx.x * 4 + orow * 2 + kh) * 2 * a.scout + a.co0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 32 * cg + 16 * j + 4 * gq;
        *(float4*)(row + c) = make_float4(s1[j][0], s1[j][1], s1[j][2], s1[j][3]);
        *(float4*)(row + a.scout + c) = make_float4(s2[j][0], s2[j][1], s2[j][2], s2[j][3]);
      }
    }
  }
}

// Two-source row ring (see conv_ring2_kernel): x0 / x1 = the two 64-channel sources (for one
// 128-channel tensor: its two halves), 64 outputs, 3x3, W % 64 == 0, even H. cout_total / co0: the
// launch computes output channels co0 .. co0 + 63 of a cout_total-channel conv (w, y, escale / eshift
// already offset by the caller; the stats rows are [rows][2][cout_total], this launch's 64 columns
// at co0). Returns the stats rows written (grid * 4), or -1 when not applicable.
extern "C" int rdp_conv_ring2(const void* x0, long xbytes0, int pitch0, const void* x1, long xbytes1, int pitch1,
                              const void* w, long wbytes, int ldw, void* y, long ybytes, int ypitch, float* stats,
                              int N, int H, int W, const float* escale, const float* eshift, int erelu, int max_blocks,
                              int cout_total, int co0, hipStream_t s) {
  if (W % 64 || H % 2 || ldw < 1152 || ypitch % 8 || pitch0 % 8 || pitch1 % 8) return -1;
  if (xbytes0 >= (1l << 31) || xbytes1 >= (1l << 31) || ybytes >= (1l << 31) || wbytes >= (1l << 31)) return -1;
  if ((escale == nullptr) != (eshift == nullptr)) return -1;
  Ring2Args a;
  a.x0 = (const u16*)x0; a.x1 = (const u16*)x1;
  a.xbytes0 = (uint32_t)xbytes0; a.xbytes1 = (uint32_t)xbytes1; a.pitch0 = pitch0; a.pitch1 = pitch1;
  a.w = (const u16*)w; a.wbytes = (uint32_t)wbytes; a.ldw = ldw;
  a.y = (u16*)y; a.ybytes = (uint32_t)ybytes; a.ypitch = ypitch;
  a.stats = stats; a.escale = escale; a.eshift = eshift; a.erelu = erelu;
  if (cout_total < 64 || co0 < 0 || co0 + 64 > cout_total) return -1;
  a.scout = cout_total; a.co0 = co0;
  a.H = H; a.W = W; a.WS = W / 64;
  a.nrows = N * a.WS * H;
  a.npairs = a.nrows / 2;
  const int blocks = std::max(1, std::min(max_blocks > 0 ? max_blocks : 256, a.npairs));
  a.pairs_per_block = (a.npairs + blocks - 1) / blocks;
  const int grid = (a.npairs + a.pairs_per_block - 1) / a.pairs_per_block;
  const FastDiv fh = make_fastdiv((uint32_t)H), fs = make_fastdiv((uint32_t)a.WS);
  a.fh_m = fh.m; a.fh_s = fh.s; a.fs_m = fs.m; a.fs_s = fs.s;
  hipLaunchKernelGGL(conv_ring2_kernel, dim3(grid), dim3(512), 0, s, a);
  return grid * 4;
}
