// Tile table of the halo-staged 3x3 convolution kernels (conv_halo.hip, conv_hx32.hip); built on the host
// by ops/halo.py (44 int32 per tile).
#pragma once

constexpr int HX_BOX = 4;      // boxes per tile
constexpr int HX_HMAX = 448;   // halo pixels per tile (per 32-ch chunk)
constexpr int HX_PB = 256;     // output pixel slots per tile

struct HaloBox {
  int sbeg;       // first output slot of the box inside the tile
  int hoff;       // first halo pixel of the box inside the halo image
  int in_base;    // input pixel index of (y, x) = (0, 0) of this image / level
  int out_base;   // output row index m of (0, 0) of this image / level
  int H, W;       // level extent
  int y0, x0;     // top-left output pixel of the box
  int R, C;       // box rows / columns
};
struct HaloTile {
  int nbox, nslot, nhalo, pad;
  HaloBox b[HX_BOX];
};
static_assert(sizeof(HaloTile) == 176, "host layout (ops/halo.py) is 44 int32 per tile");

// index of the box holding value v (boxes are sorted by both sbeg and hoff; fields come from SGPRs)
#define HX_SELECT(FIELD, v)                                                              \
  int sel = 0;                                                                           \
  _Pragma("unroll") for (int t_ = 1; t_ < HX_BOX; ++t_) if (t_ < T.nbox && (v) >= T.b[t_].FIELD) sel = t_;
