// Geometry of one implicit-GEMM convolution launch (shared by host and device code).
#pragma once

namespace dm {

constexpr int MAXTAPS = 64;

struct ConvGeom {
  int N, H, W, C;            // input tensor NHWC; C % 8 == 0 and C/8 a power of two
  int lgC8;                  // log2(C / 8)
  int Hg, Wg;                // GEMM rows: m = (n*Hg + y)*Wg + x
  int isy, isx;              // input coordinate = (y*isy + dy_t, x*isx + dx_t)
  int OH, OW, OC;            // output tensor (NHWC, channel count OC)
  int osy, osx, oy0, ox0;    // output coordinate = (y*osy + oy0, x*osx + ox0)
  // tap grid: t = th*ntw + tw, th < nth, tw < ntw
  int nth, ntw;
  int dy0, dys, dx0, dxs;    // dy_t = dy0 + th*dys, dx_t = dx0 + tw*dxs
  int kh0, khs, kw0, kws, KW;// packed-weight tap = (kh0 + th*khs)*KW + (kw0 + tw*kws)
  int Ncols;                 // output channels of the GEMM
  int wK;                    // packed weight row length (elements) = KH*KW*C
  long long M;               // N*Hg*Wg
  int K;                     // ntaps*C
  // magic-number division by Wg and Hg (m < 2^31): q = (umulhi(n, mul) + n) >> shr
  unsigned wg_mul, wg_shr, hg_mul, hg_shr;
};

// BatchNorm-backward sums fused into a dgrad epilogue.  The dgrad output is the upstream
// gradient `dout` of the BN that produced this conv's input; with y (that BN's input, same
// NHWC layout as the dgrad output) the epilogue reduces per channel
//     Σ dz,  Σ dz·(y - mean)·invstd       dz = dout masked by the BN's ReLU
// into the stats slab rows (the layout of the forward statistics), so the BN backward
// needs no separate reduction pass over dout and y.  mode: 0 no ReLU, 1 mask out > 0
// (block output with residual), 2 mask y*sc + sh > 0, 4 the forward's 1-bit (out > 0) mask
// (bit j of byte i: channel j of 8-channel chunk i).  y == nullptr: disabled.
struct BnBwdEpi {
  const unsigned short* y;
  const unsigned short* out;
  const float* mean;
  const float* invstd;
  const float* sc;
  const float* sh;
  int mode;
  const unsigned char* mask;
};

// several geometries for one launch (selected by blockIdx.z)
struct ConvGeomSet {
  ConvGeom g[4];
  BnBwdEpi bnb;
  static ConvGeomSet one(const ConvGeom& g0, const BnBwdEpi* b = nullptr) {
    ConvGeomSet s{};
    s.g[0] = g0;
    if (b) s.bnb = *b;
    return s;
  }
};

inline void fastdiv_init(unsigned d, unsigned& mul, unsigned& shr) {
  unsigned l = 0;
  while ((1u << l) < d) ++l;
  mul = (unsigned)((((unsigned long long)1 << 32) * ((1ull << l) - d)) / d + 1);
  shr = l;
}
inline void geom_finalize(ConvGeom& g) {
  fastdiv_init((unsigned)g.Wg, g.wg_mul, g.wg_shr);
  fastdiv_init((unsigned)g.Hg, g.hg_mul, g.hg_shr);
}

}  // namespace dm
