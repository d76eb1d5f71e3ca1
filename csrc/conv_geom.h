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
  // optional 1-bit mask of the epilogue's ADD operand (bit j of byte i = element 8i + j of the
  // NHWC output): the identity-skip gradient dres = dout * mask is added without ever being
  // materialised (0 = plain ADD)
  const unsigned char* addm;
};

// several geometries for one launch (selected by blockIdx.z)
struct ConvGeomSet {
  ConvGeom g[4];
  static ConvGeomSet one(const ConvGeom& g0) {
    ConvGeomSet s{};
    s.g[0] = g0;
    return s;
  }
};

// A second K segment appended to one geometry of a ConvGeomSet launch: after the geometry's
// own taps, the block accumulates X2[pixel] . W2 over C2 more channels at the SAME GEMM row
// pixel (tap offset 0).  The stride-2 block's 1x1/s2/p0 projection has exactly the pixel map
// of the 3x3/s2/p1 conv's parity class (0,0) centre tap, so its data gradient joins that
// class's K loop and the block output gradient is written once (no accumulate pass).
struct DgradSeg2 {
  const void* X2;      // bf16 [N][H][W][C2] (the geometry's input grid)
  const void* W2;      // bf16 [Ncols][C2]
  unsigned x2bytes, w2bytes;
  int C2;              // channels of X2 (multiple of 64)
  int z;               // geometry index (blockIdx.z) that takes the segment
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
