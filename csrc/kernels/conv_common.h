// Shared pieces of the implicit-GEMM convolution kernels (forward/dgrad and wgrad).
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define MXR_MAXLEV 5

struct ConvGeom {
  int nlev;
  int H[MXR_MAXLEV], W[MXR_MAXLEV], Ho[MXR_MAXLEV], Wo[MXR_MAXLEV];
  int in_off[MXR_MAXLEV];      // pixel offset of level l inside one image's input block
  int mstart[MXR_MAXLEV + 1];  // output pixel offset of level l inside one image's output block
  int in_img, out_img;         // pixels per image (input / output)
  int stride, pt, pl, kh, kw;
  int cin, cout;
  long long M;                 // batch * out_img
  int ostride, oH, oW;         // strided output scatter (single level): dst = (oy*os + ooy, ox*os + oox) in oH x oW
  int ooy, oox;                // scatter phase (sub-pixel stride-2 data gradient); 0 = the gap-zeroing phase
};


template <int NS>
struct PixSlot {
  int base[NS];   // b*in_img + in_off[l]  (-1 = invalid row)
  int iy0[NS], ix0[NS], Hl[NS], Wl[NS];
};

static __device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// The same 16-B-per-lane LDS-DMA issued as inline asm: the compiler tracks no pending LDS-DMA write for
// it.  A TRACKED one makes the compiler put an s_waitcnt vmcnt(0) in front of the next ds_read_b64_tr_b16
// (that builtin carries no alias information), i.e. every transposed-read phase waits for ALL DMA in flight.
// Only for kernels whose own counted vmcnt waits + barriers order the LDS reads after the data lands.
static __device__ __forceinline__ void glds16_asm(const void* src, const void* lds_base) {
  // (readfirstlane: the base is wave-uniform by contract; an "s" operand the compiler cannot prove uniform
  // would be handed a VGPR)
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}

// glds16_asm with the LDS byte address already in hand (lds_addr(smem) + a uniform offset): no generic ->
// LDS pointer conversion (its null check is ~8 scalar instructions per piece)
static __device__ __forceinline__ void glds16_m0(const void* src, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src),
               "s"(__builtin_amdgcn_readfirstlane(m0)) : "memory", "m0");
}

static __device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

static __device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7, i = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// The pyramid level of output pixel q of an image, its fields picked by a select chain over the
// statically indexed levels.  (Indexing the by-value ConvGeom's arrays with a computed level makes
// hipcc read them with vector loads from the kernel-argument segment, each waited on with vmcnt(0):
// microseconds per decoded row.)
struct LevelSel {
  int mstart, wo, in_off, H, W;
};

static __device__ __forceinline__ void select_level(const ConvGeom& g, int q, LevelSel& s) {
  s.mstart = g.mstart[0];
  s.wo = g.Wo[0];
  s.in_off = g.in_off[0];
  s.H = g.H[0];
  s.W = g.W[0];
#pragma unroll
  for (int t = 1; t < MXR_MAXLEV; ++t) {
    const bool in = t < g.nlev && q >= g.mstart[t];
    s.mstart = in ? g.mstart[t] : s.mstart;
    s.wo = in ? g.Wo[t] : s.wo;
    s.in_off = in ? g.in_off[t] : s.in_off;
    s.H = in ? g.H[t] : s.H;
    s.W = in ? g.W[t] : s.W;
  }
}

// Decode an output row m -> (pixel base of its image/level in the input, iy0, ix0, H, W).
static __device__ __forceinline__ void decode_row(const ConvGeom& g, long long m, int& base, int& iy0, int& ix0, int& Hl, int& Wl,
                                           int& b, int& oy, int& ox) {
  b = (int)(m / g.out_img);
  const int q = (int)(m - (long long)b * g.out_img);
  LevelSel s;
  select_level(g, q, s);
  const int loc = q - s.mstart;
  oy = loc / s.wo;
  ox = loc - oy * s.wo;
  base = b * g.in_img + s.in_off;
  iy0 = oy * g.stride - g.pt;
  ix0 = ox * g.stride - g.pl;
  Hl = s.H;
  Wl = s.W;
}

// Exact integer division n / d for 0 <= n < 2^24 via the hardware fp32 reciprocal (v_rcp_f32) and a
// +-1 fix-up -- replaces the ~40-instruction integer-division sequence on the per-step decode path.
static __device__ __forceinline__ int fdiv(int n, int d) {
  int q = __float2int_rz((float)n * __builtin_amdgcn_rcpf((float)d));
  const int r = n - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

// decode_row for m < 2^24 (used on the per-step hot path of the wgrad kernel)
static __device__ __forceinline__ void decode_row_fast(const ConvGeom& g, int m, int& base, int& iy0, int& ix0,
                                                       int& Hl, int& Wl) {
  const int b = fdiv(m, g.out_img);
  const int q = m - b * g.out_img;
  LevelSel s;
  select_level(g, q, s);
  const int loc = q - s.mstart;
  const int oy = fdiv(loc, s.wo);
  const int ox = loc - oy * s.wo;
  base = b * g.in_img + s.in_off;
  iy0 = oy * g.stride - g.pt;
  ix0 = ox * g.stride - g.pl;
  Hl = s.H;
  Wl = s.W;
}

// Sweep epilogue of 8 consecutive outputs v (fp32) at element offset off: + residual R (at roff: the
// GEMM row, which differs from off under a strided scatter), + the existing output Yacc (accumulate),
// ReLU, then the relu-gradient mask Mk (keep where Mk > 0).  The (up to three)
// 16-B loads are issued together before any is used -- one memory latency per chunk instead of three.
//
// Mk with pointer bit 0 set is a BITMASK instead of the bf16 activation: byte (off >> 3) holds channels
// off .. off + 7 (bit j: channel off + j > 0 as a bf16), 1/16 of the activation's bytes.  A forward epilogue
// WITH relu writes it (the mask of its own output, for the consumer's data gradient); a data-gradient
// epilogue (no relu) reads it.  off is always a multiple of 8 here (16-B chunks of a cout % 8 == 0 row).
static __device__ __forceinline__ bool mk_bits(const bf16_t* Mk) { return ((uintptr_t)Mk & 1) != 0; }
static __device__ __forceinline__ uint8_t* mk_byte(const bf16_t* Mk, long long off) {
  return (uint8_t*)((uintptr_t)Mk & ~(uintptr_t)1) + (off >> 3);
}
// bit j set where bf16(v[j]) > 0 (the value the caller stores)
static __device__ __forceinline__ uint32_t mk_pack(const float (&v)[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) b |= (uint32_t)(__builtin_bit_cast(short, f2bf(v[j])) > 0) << j;
  return b;
}

// the epilogue operands of 8 consecutive output channels (residual, previous output, relu-gradient mask),
// loaded by epi_load8 ahead of their use so several chunks' loads are in flight together
// (bitmask Mk: m.x = the mask byte, m.y / m.z = the byte index for the writing form)
struct Epi8 {
  uint4 r, y, m;
};

static __device__ __forceinline__ void epi_load8(Epi8& e, const bf16_t* R, long long roff, const bf16_t* Yacc,
                                                 const bf16_t* Mk, long long off) {
  e.r = e.y = e.m = make_uint4(0u, 0u, 0u, 0u);
  if (R) e.r = *reinterpret_cast<const uint4*>(R + roff);
  if (Yacc) e.y = *reinterpret_cast<const uint4*>(Yacc + off);
  if (Mk) {
    if (mk_bits(Mk)) e.m = make_uint4((uint32_t)*mk_byte(Mk, off), (uint32_t)off, (uint32_t)(off >> 32), 0u);
    else e.m = *reinterpret_cast<const uint4*>(Mk + off);
  }
}

// the mask step of both epilogue forms (bf16 words m4, or the bitmask byte / written byte)
static __device__ __forceinline__ void epi_mask8(float (&v)[8], const bf16_t* Mk, const uint4 mm, long long off,
                                                 bool relu) {
  if (mk_bits(Mk)) {
    if (relu) {
      *mk_byte(Mk, off) = (uint8_t)mk_pack(v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (!((mm.x >> j) & 1u)) v[j] = 0.f;
    }
    return;
  }
  const uint32_t m4[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!(bf2f((bf16_t)(m4[q] & 0xffff)) > 0.f)) v[2 * q] = 0.f;
    if (!(bf2f((bf16_t)(m4[q] >> 16)) > 0.f)) v[2 * q + 1] = 0.f;
  }
}

static __device__ __forceinline__ void epi_apply8(float (&v)[8], const Epi8& e, const bf16_t* R, const bf16_t* Yacc,
                                                  const bf16_t* Mk, bool relu) {
  const uint4 rr = e.r, yy = e.y;
  const uint32_t r4[4] = {rr.x, rr.y, rr.z, rr.w}, y4[4] = {yy.x, yy.y, yy.z, yy.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (R) {
      v[2 * q] += bf2f((bf16_t)(r4[q] & 0xffff));
      v[2 * q + 1] += bf2f((bf16_t)(r4[q] >> 16));
    }
    if (Yacc) {
      v[2 * q] += bf2f((bf16_t)(y4[q] & 0xffff));
      v[2 * q + 1] += bf2f((bf16_t)(y4[q] >> 16));
    }
    if (relu) {
      v[2 * q] = fmaxf(v[2 * q], 0.f);
      v[2 * q + 1] = fmaxf(v[2 * q + 1], 0.f);
    }
  }
  if (Mk) epi_mask8(v, Mk, e.m, (long long)(((unsigned long long)e.m.z << 32) | e.m.y), relu);
}

static __device__ __forceinline__ void epi_sweep8(float (&v)[8], const bf16_t* R, long long roff, const bf16_t* Yacc,
                                                  const bf16_t* Mk, long long off, bool relu) {
  uint4 rr = make_uint4(0u, 0u, 0u, 0u), yy = rr, mm = rr;
  if (R) rr = *reinterpret_cast<const uint4*>(R + roff);
  if (Yacc) yy = *reinterpret_cast<const uint4*>(Yacc + off);
  if (Mk) {
    if (mk_bits(Mk)) mm.x = relu ? 0u : (uint32_t)*mk_byte(Mk, off);
    else mm = *reinterpret_cast<const uint4*>(Mk + off);
  }
  const uint32_t r4[4] = {rr.x, rr.y, rr.z, rr.w}, y4[4] = {yy.x, yy.y, yy.z, yy.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (R) {
      v[2 * q] += bf2f((bf16_t)(r4[q] & 0xffff));
      v[2 * q + 1] += bf2f((bf16_t)(r4[q] >> 16));
    }
    if (Yacc) {
      v[2 * q] += bf2f((bf16_t)(y4[q] & 0xffff));
      v[2 * q + 1] += bf2f((bf16_t)(y4[q] >> 16));
    }
    if (relu) {
      v[2 * q] = fmaxf(v[2 * q], 0.f);
      v[2 * q + 1] = fmaxf(v[2 * q + 1], 0.f);
    }
  }
  if (Mk) epi_mask8(v, Mk, mm, off, relu);
}

// XOR swizzles of the 16-B chunk index for LDS tiles read with ds_read_b64_tr_b16: conflict-free
// for the 4-row x 16-column blocks of two 16-lane groups 8 rows apart (see conv_wgrad.hip).
static __device__ __forceinline__ int swz8(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
static __device__ __forceinline__ int swz16(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }
