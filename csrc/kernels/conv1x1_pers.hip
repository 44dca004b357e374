// Persistent streaming 1x1 / stride-1 convolution (forward, and the data gradient of a 1x1 / stride-1 conv,
// which is the same GEMM with the transposed weights), NHWC bf16 on the 32x32x16 MFMA, for gfx950.
//
// The backbone's bottleneck 1x1 layers and the FPN laterals (256 -> 1024, 1024 -> 256,
// 512 -> 2048, ... at 67k - 1.07M pixels, built at /root/reference/train.py:91) are short-K GEMMs whose bytes
// (residual, output, relu mask) outweigh their MACs: conv_pipe.hip runs them at 2.9 - 3.4 TB/s because every
// block pays its ring's fill latency at the start (a K = 256 tile has 8 sub-stages) and drains all its loads
// before its epilogue.  Here one block per CU walks its tiles with ONE continuous LDS-DMA stream:
//
// * tile = 128 output channels x 128 pixels, 8 waves as 2 (co) x 4 (px), each 64 x 32 = 2 x 1 accumulators
//   of 32 x 32; K in 32-deep stages (64-B rows), a 4-slot ring filled THREE stages ahead -- across tile
//   boundaries, so the next tile's first stages land while this one finishes and runs its epilogue;
// * the epilogue operands (residual, previous output, relu-gradient mask or its bits, bias) come in by
//   LDS-DMA too, two stages before the tile's last one, into a per-wave area where each lane later reads back
//   the bytes it fetched; the 16-B stores go straight from the accumulators (v_permlane32_swap pairs give each
//   lane 8 consecutive channels: conv_hx32.hip's epilogue);
// * every global load is an opaque LDS-DMA and every wait a counted vmcnt: each wave issues the same number of
//   vector-memory operations per stage (2 pieces), per epilogue (NE DMA pieces, NS stores: chunks outside the
//   tensor load the zero page and store into a scratch line instead of being skipped), so no wait drains the
//   stream -- and the compiler, which sees no load of its own, inserts none (a compiler-visible epilogue load is
//   the youngest op it knows, so its use costs a vmcnt(0) that drains the next tile's prefetch: measured, the
//   first form of this kernel ran 0.70-0.97x the best pipe kernel);
// * LDS images: 16-B chunk c of row r at 16 (c ^ (r >> 2 & 3)) -- the 32x32x16 operand read of any
//   32 consecutive rows hits 16 distinct bank slots per 16-lane group (conv_hx32.hip's HL = 1 layout);
//   the swizzle is applied at the DMA source, the image stays lane-linear;
// * tiles are assigned XCD-major (xcd_remap): the channel slices of a pixel tile run on one XCD at the same
//   time and share its X rows in L2.
//
// EPI (compile-time epilogue form): 1 residual R, 2 accumulate into Y, 4 relu-gradient mask read (bf16
// activation; with 32: the BitMask, pointer bit 0), 8 relu-mask bits WRITE (forward with relu), 16 bias.
#include "conv_common.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace {

constexpr int Q_NW = 8, Q_BM = 128, Q_BN = 128, Q_NS = 4;
constexpr int Q_WPX = 4;                             // wave grid: 2 (co) x 4 (px)
constexpr int Q_WTC = 64, Q_WTP = 32;                // 64 co x 32 px per wave
constexpr int Q_TI = 2;                              // 32 x 32 accumulators per wave (co)
constexpr int Q_STAGE = (Q_BN + Q_BM) * 64;          // 16 KiB per stage
constexpr int Q_D = (Q_BN + Q_BM) / 16 / Q_NW;       // 1-KiB DMA pieces per wave per stage (2)
constexpr int Q_NCH = Q_TI * 2;                      // 16-B output chunks per lane per tile
constexpr int Q_EOFF = Q_NS * Q_STAGE;               // epilogue operand area behind the ring
static_assert(Q_D * 16 * Q_NW == Q_BN + Q_BM, "DMA pieces split evenly over the waves");

template <int EPI>
struct QEpi {
  static constexpr bool R = (EPI & 1) != 0, Y = (EPI & 2) != 0, MR = (EPI & 4) != 0, MW = (EPI & 8) != 0,
                        B = (EPI & 16) != 0, BITS = (EPI & 32) != 0;
  static constexpr bool MB = MR && !BITS;                             // bf16 mask (16 B per chunk)
  static constexpr bool MBITS = MR && BITS;                           // bitmask read (one 4-B word per chunk)
  static constexpr int N16 = (int)R + (int)Y + (int)MB;               // 16-B operands per chunk
  static constexpr int NE = Q_NCH * (N16 + (MBITS ? 1 : 0)) + (B ? 1 : 0);   // DMA ops per lane per tile
  static constexpr int NS = Q_NCH * (1 + (int)MW);                    // stores per lane per tile
  // per wave: N16 x NCH KiB of 16-B pieces, NCH x 256 B of bitmask words, 1 KiB for the bias piece
  static constexpr int WAREA = N16 * Q_NCH * 1024 + (MBITS ? Q_NCH * 256 : 0) + (B ? 1024 : 0);
  static constexpr int LDS = Q_EOFF + Q_NW * WAREA;
};

template <int N>
__device__ __forceinline__ void q_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void q_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 4-B-per-lane LDS-DMA (lane l writes LDS base + 4 l), opaque like glds16_asm
__device__ __forceinline__ void glds4_asm(const void* src, const void* lds_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ int q_off(int r, int c) { return (r << 6) + ((c ^ ((r >> 2) & 3)) << 4); }

// DS (dual source, a projection block's branch2c + branch1 in one GEMM; conv_pipe.hip DualSrc): K stages below
// q.k1 read row m of X / Wt (channel stride k1), the rest row m's pixel (b, oy*s, ox*s) of X2 (H x W grid, channel
// stride K - k1) and W2.
struct QDual {
  const bf16_t* x2;
  const bf16_t* w2;
  int k1, H, W, s, Ho, Wo;
};

template <int EPI, int DS = 0>
__global__ __launch_bounds__(Q_NW * 64, 1) void conv1x1_pers_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt, const float* __restrict__ bias,
    const bf16_t* __restrict__ R, const bf16_t* __restrict__ Mk, bf16_t* __restrict__ Y,
    const bf16_t* __restrict__ zpage, bf16_t* __restrict__ trash, int M, int N, int K, int relu, int tiles_n,
    int ntiles, QDual qd) {
  using E = QEpi<EPI>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wco = wave / Q_WPX, wpx = wave % Q_WPX;
  const int nks = K >> 5;                          // stages per tile (>= 3)
  const int grid = gridDim.x;
  const int first = xcd_remap(blockIdx.x, grid);
  const int my_tiles = first < ntiles ? (ntiles - 1 - first) / grid + 1 : 0;   // tiles first, first + grid, ...
  const long long total = (long long)my_tiles * nks;   // stages of the block's stream

  // ---- DMA: piece p of a stage = 16 rows of 64 B; wave w issues piece w (W rows w * 16 ..) and piece w + 8
  // (X rows w * 16 ..).  Lane L writes LDS bytes 16 L of its piece = row L / 4, physical chunk L & 3, so it
  // fetches logical chunk (L & 3) ^ ((L >> 4) & 3) of that row (the swizzle at the source).
  const int prow = lane >> 2;
  const int pchunk = (lane & 3) ^ ((lane >> 4) & 3);
  const bf16_t* wsrc = nullptr;      // W row of this lane's piece (tile of the issue cursor), nullptr = zeros
  const bf16_t* xsrc = nullptr;
  const bf16_t* wsrc2 = nullptr;     // DS: the second sources, offset so that + ko (ko >= k1) addresses them
  const bf16_t* xsrc2 = nullptr;
  auto cursor_tile = [&](int ti) {   // the issue cursor enters the block's ti-th tile
    const int t = first + ti * grid;
    const int tn = t % tiles_n, tm = t / tiles_n;
    const int co = tn * Q_BN + wave * 16 + prow;
    const long long m = (long long)tm * Q_BM + wave * 16 + prow;
    if constexpr (DS) {
      const int k2 = K - qd.k1;
      wsrc = co < N ? Wt + (long long)co * qd.k1 + pchunk * 8 : nullptr;
      wsrc2 = co < N ? qd.w2 + (long long)co * k2 - qd.k1 + pchunk * 8 : nullptr;
      xsrc = m < M ? X + m * qd.k1 + pchunk * 8 : nullptr;
      if (m < M) {
        const int img = qd.Ho * qd.Wo;
        const int b = (int)(m / img), q = (int)(m - (long long)b * img);
        const int oy = q / qd.Wo, ox = q - oy * qd.Wo;
        xsrc2 = qd.x2 + ((long long)(b * qd.H + oy * qd.s) * qd.W + ox * qd.s) * k2 - qd.k1 + pchunk * 8;
      } else {
        xsrc2 = nullptr;
      }
    } else {
      wsrc = co < N ? Wt + (long long)co * K + pchunk * 8 : nullptr;
      xsrc = m < M ? X + m * K + pchunk * 8 : nullptr;
    }
  };
  long long iss = 0;                 // next stage of the stream to issue
  int iss_tile = 0, iss_k = 0;
  if (my_tiles > 0) cursor_tile(0);
  auto issue = [&]() {
    char* base = smem + (int)(iss % Q_NS) * Q_STAGE;
    const bool live = iss < total;   // past the stream's end: same shape, the zero page into the free slot
    const int ko = iss_k * 32;
    const bf16_t* ws = wsrc;
    const bf16_t* xs = xsrc;
    if constexpr (DS) {
      if (ko >= qd.k1) {
        ws = wsrc2;
        xs = xsrc2;
      }
    }
    const void* a0 = (live && ws) ? (const void*)(ws + ko) : (const void*)zpage;
    const void* a1 = (live && xs) ? (const void*)(xs + ko) : (const void*)zpage;
    glds16_asm(a0, base + wave * 1024);
    glds16_asm(a1, base + Q_BN * 64 + wave * 1024);
    ++iss;
    if (++iss_k == nks) {
      iss_k = 0;
      if (++iss_tile < my_tiles) cursor_tile(iss_tile);
    }
  };

  // ---- fragment reads (lane constants inside a stage slot)
  const int fh = lane >> 5;
  int aoff[Q_TI][2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < Q_TI; ++i) aoff[i][kk] = q_off(wco * Q_WTC + i * 32 + (lane & 31), 2 * kk + fh);
    boff[kk] = Q_BN * 64 + q_off(wpx * Q_WTP + (lane & 31), 2 * kk + fh);
  }

  // ---- epilogue operands: chunk c = (i, qp) of this lane = pixel m, 8 channels from cg
  char* ew = smem + Q_EOFF + wave * E::WAREA;    // this wave's area
  auto chunk_pos = [&](int t, int c, long long& m, int& cg) {
    const int i = c >> 1, qp = c & 1;
    const int tn = t % tiles_n, tm = t / tiles_n;
    m = (long long)tm * Q_BM + wpx * Q_WTP + (lane & 31);
    cg = tn * Q_BN + wco * Q_WTC + i * 32 + 16 * qp + 8 * fh;
    return m < M && cg < N;
  };
  auto op16 = [&](int t, const bf16_t* base, int o) {
#pragma unroll
    for (int c = 0; c < Q_NCH; ++c) {
      long long m;
      int cg;
      const bool ok = chunk_pos(t, c, m, cg);
      glds16_asm(ok ? (const void*)(base + m * N + cg) : (const void*)zpage, ew + (o * Q_NCH + c) * 1024);
    }
  };
  auto issue_epi = [&](int t) {
    if constexpr (E::R) op16(t, R, 0);
    if constexpr (E::Y) op16(t, Y, (int)E::R);
    if constexpr (E::MB) op16(t, Mk, (int)E::R + (int)E::Y);
    if constexpr (E::MBITS) {
      // the bitmask byte of a chunk sits in the 4-B word at (its address & ~3)
#pragma unroll
      for (int c = 0; c < Q_NCH; ++c) {
        long long m;
        int cg;
        const bool ok = chunk_pos(t, c, m, cg);
        const uintptr_t b = ok ? (uintptr_t)mk_byte(Mk, m * N + cg) : (uintptr_t)zpage;
        glds4_asm((const void*)(b & ~(uintptr_t)3), ew + E::N16 * Q_NCH * 1024 + c * 256);
      }
    }
    if constexpr (E::B) {
      // lanes 0-15: 4 of this wave's 64 channels; the others (and channels past N) read the zero page
      const int co = (t % tiles_n) * Q_BN + wco * Q_WTC + 4 * (lane & 15);
      glds16_asm((lane < 16 && co < N) ? (const void*)(bias + co) : (const void*)zpage, ew + E::WAREA - 1024);
    }
  };

  f32x16 acc[Q_TI];

  // per-stage wait: the stage's own DMA; younger = the next two stages' DMA, plus the previous tile's stores
  // (steps 0-2 of a tile after the first) and this tile's epilogue DMA (the last two steps)
  auto wait_stage = [&](int s, bool after_first) {
    const bool ws = after_first && s <= 2;
    const bool we = s >= nks - 2;
    constexpr int D2 = 2 * Q_D;
    if (ws && we) q_vm_wait<D2 + E::NS + E::NE>();
    else if (ws) q_vm_wait<D2 + E::NS>();
    else if (we) q_vm_wait<D2 + E::NE>();
    else q_vm_wait<D2>();
  };

  if (my_tiles > 0) {
    issue();
    issue();
    issue();
  }
  for (int ti = 0; ti < my_tiles; ++ti) {
    const int t = first + ti * grid;
#pragma unroll
    for (int i = 0; i < Q_TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    // one K stage: wait for its DMA, barrier, issue the stage three ahead, (the tile's epilogue DMA), fragment
    // reads + 4 MFMAs.  The epilogue-DMA step is its own call, not a branch inside the loop.
    auto step = [&](int s, bool epi) {
      const int slot = (int)(((long long)ti * nks + s) % Q_NS);
      wait_stage(s, ti > 0);
      q_sync();                      // every wave's DMA of this stage landed; every wave done with slot s - 1
      issue();                       // stage + 3 into slot s - 1
      if (epi) issue_epi(t);
      const char* sb = smem + slot * Q_STAGE;
      bf16x8 fa[2][Q_TI], fb[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < Q_TI; ++i) fa[kk][i] = *reinterpret_cast<const bf16x8*>(sb + aoff[i][kk]);
        fb[kk] = *reinterpret_cast<const bf16x8*>(sb + boff[kk]);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < Q_TI; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk][i], fb[kk], acc[i], 0, 0, 0);
    };
#pragma nounroll
    for (int s = 0; s < nks - 3; ++s) step(s, false);
    step(nks - 3, true);
    step(nks - 2, false);
    step(nks - 1, false);

    // ---- epilogue: this tile's operands (DMA'd two stages ago) have landed once the two stages issued after
    // them are the only younger operations; each lane reads back exactly the bytes its own DMA wrote
    q_vm_wait<2 * Q_D>();
#pragma unroll
    for (int i = 0; i < Q_TI; ++i) {
      // lanes 0-31 hold channels 8 q + 0..3, lanes 32-63 8 q + 4..7 (q = 0..3) of pixel lane % 32: two swaps
      // per channel pair (q, q + 1) give every lane 8 consecutive channels 16 qp + 8 fh + 0..7
      f32x16 a = acc[i];
#pragma unroll
      for (int qp = 0; qp < 2; ++qp)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[8 * qp + r]),
                                                           __float_as_uint(a[8 * qp + 4 + r]), false, false);
          a[8 * qp + r] = __uint_as_float(sw[0]);
          a[8 * qp + 4 + r] = __uint_as_float(sw[1]);
        }
#pragma unroll
      for (int qp = 0; qp < 2; ++qp) {
        const int c = (i << 1) | qp;
        long long m;
        int cg;
        const bool ok = chunk_pos(t, c, m, cg);
        const long long off = m * N + cg;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = a[8 * qp + e];
        if constexpr (E::B) {
          // the wave's 64 bias values sit in lanes 0-15's 16 B of the bias piece
          const float* bl = reinterpret_cast<const float*>(ew + E::WAREA - 1024);
          const int cl = i * 32 + 16 * qp + 8 * fh;   // channel inside the wave's 64
          const float4 b0 = *reinterpret_cast<const float4*>(bl + cl);
          const float4 b1 = *reinterpret_cast<const float4*>(bl + cl + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
          v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        auto add16 = [&](int o) {
          const uint4 rr = *reinterpret_cast<const uint4*>(ew + (o * Q_NCH + c) * 1024 + 16 * lane);
          const uint32_t r4[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] += bf2f((bf16_t)(r4[q] & 0xffff));
            v[2 * q + 1] += bf2f((bf16_t)(r4[q] >> 16));
          }
        };
        if constexpr (E::R) add16(0);
        if constexpr (E::Y) add16((int)E::R);
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if constexpr (E::MB) {
          const uint4 mm = *reinterpret_cast<const uint4*>(ew + (((int)E::R + (int)E::Y) * Q_NCH + c) * 1024 + 16 * lane);
          const uint32_t m4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!(bf2f((bf16_t)(m4[q] & 0xffff)) > 0.f)) v[2 * q] = 0.f;
            if (!(bf2f((bf16_t)(m4[q] >> 16)) > 0.f)) v[2 * q + 1] = 0.f;
          }
        }
        if constexpr (E::MBITS) {
          const uint32_t wd = *reinterpret_cast<const uint32_t*>(ew + E::N16 * Q_NCH * 1024 + c * 256 + 4 * lane);
          const uint32_t byte = (wd >> (8 * (int)((uintptr_t)mk_byte(Mk, off) & 3))) & 0xffu;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (!((byte >> e) & 1u)) v[e] = 0.f;
        }
        uint4 ov;
        ov.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        ov.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        ov.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
        ov.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        *reinterpret_cast<uint4*>(ok ? Y + off : trash) = ov;
        if constexpr (E::MW) *(ok ? mk_byte(Mk, off) : (uint8_t*)trash + 64) = (uint8_t)mk_pack(v);
      }
    }
  }
  q_vm_wait<0>();   // the stream's trailing DMA lands before the workgroup's LDS is released
}

template <int EPI, int DS = 0>
int launch_q(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
             const void* zpage, void* trash, int M, int N, int K, int relu, int ncu, hipStream_t stream,
             QDual qd = QDual{}) {
  const int tiles_n = (N + Q_BN - 1) / Q_BN;
  const long long ntiles = (long long)((M + Q_BM - 1) / Q_BM) * tiles_n;
  if (ntiles < 1 || ntiles > 0x7fffffffLL) return -3;
  auto kern = conv1x1_pers_kernel<EPI, DS>;
  constexpr int lds = QEpi<EPI>::LDS;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  const int grid = (int)std::min<long long>(ntiles, ncu);
  kern<<<grid, Q_NW * 64, lds, stream>>>((const bf16_t*)X, (const bf16_t*)Wt, bias, (const bf16_t*)R,
                                         (const bf16_t*)Mk, (bf16_t*)Y, (const bf16_t*)zpage, (bf16_t*)trash, M, N, K,
                                         relu, tiles_n, (int)ntiles, qd);
  return (int)hipGetLastError();
}

}  // namespace

// Y (M x N) = epilogue(X (M x K) . Wt (N x K)^T): a 1x1 / stride-1 conv (forward: Wt = OHWI weights; data
// gradient: X = dY, Wt = the transposed weights).  bias: fp32 N (or null); R: residual M x N; accumulate:
// Y += result; Mk: relu-gradient mask (bf16 M x N, or a BitMask pointer with bit 0 set: read, or written when
// relu != 0).  zpage: >= 64 zero bytes; trash: >= 128 writable scratch bytes (stores of chunks outside the
// tensor go there).  Requires K % 32 == 0, K >= 96, N % 8 == 0, 16-B aligned operands, M < 2^31.
MXR_API int mxr_conv1x1_pers(const void* X, const void* Wt, const float* bias, const void* R, const void* Mk, void* Y,
                             const void* zpage, void* trash, long long M, int N, int K, int relu, int accumulate,
                             hipStream_t stream) {
  if (M < 1 || N < 8 || N % 8 || K % 32 || K < 96 || M >= (1LL << 31)) return -1;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu < 1) ncu = 256;
  }
  const bool bits = Mk != nullptr && ((uintptr_t)Mk & 1) != 0;
  int epi = (bias ? 16 : 0) | (R ? 1 : 0) | (accumulate ? 2 : 0);
  if (Mk) epi |= (bits && relu) ? 8 : (bits ? (4 | 32) : 4);
  const int m = (int)M;
#define Q_CASE(E_)                                                                                          \
  case E_:                                                                                                  \
    return launch_q<E_>(X, Wt, bias, R, Mk, Y, zpage, trash, m, N, K, relu, ncu, stream);
  switch (epi) {
    Q_CASE(0) Q_CASE(2) Q_CASE(4) Q_CASE(6) Q_CASE(36) Q_CASE(38) Q_CASE(16) Q_CASE(17) Q_CASE(20) Q_CASE(24)
    Q_CASE(25)
    default: return -2;
  }
#undef Q_CASE
}

// Dual-source form (QDual): Y (M x N) = relu([X (M x k1) | X2 strided (M x (K - k1))] . [Wt (N x k1) | W2 (N x (K - k1))]^T
// + bias), the fused branch2c + branch1 + add + relu of a projection block; Mk: the output's relu bits (pointer bit 0
// set) or null.  X2: [*, H, W, K - k1] read at (oy * s, ox * s) of the Ho x Wo output grid.  k1, K - k1 % 32 == 0.
MXR_API int mxr_conv1x1_pers_dual(const void* X, const void* X2, const void* Wt, const void* W2, const float* bias,
                                  const void* Mk, void* Y, const void* zpage, void* trash, long long M, int N, int K,
                                  int k1, int H, int W, int s, int Ho, int Wo, hipStream_t stream) {
  if (M < 1 || N < 8 || N % 8 || K % 32 || K < 96 || k1 % 32 || (K - k1) % 32 || k1 < 32 || k1 >= K ||
      M >= (1LL << 31) || bias == nullptr)
    return -1;
  if (s < 1 || (Ho - 1) * s >= H || (Wo - 1) * s >= W || M % ((long long)Ho * Wo) != 0) return -4;
  if (Mk != nullptr && ((uintptr_t)Mk & 1) == 0) return -5;    // only the written bitmask
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu < 1) ncu = 256;
  }
  const QDual qd{(const bf16_t*)X2, (const bf16_t*)W2, k1, H, W, s, Ho, Wo};
  if (Mk) return launch_q<24, 1>(X, Wt, bias, nullptr, Mk, Y, zpage, trash, (int)M, N, K, 1, ncu, stream, qd);
  return launch_q<16, 1>(X, Wt, bias, nullptr, nullptr, Y, zpage, trash, (int)M, N, K, 1, ncu, stream, qd);
}
