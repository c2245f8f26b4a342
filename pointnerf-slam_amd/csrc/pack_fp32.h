// pack_fp32.h -- element idx of the fp32 MFMA weight image (k_pack; pnr_internal.h layout), shared by
// mlp.hip's k_pack and the split-precision packer's first stage (mlp16_pack.hip k_pack_stage1).
#pragma once
#include "dev_common.h"

namespace pnr {

// (32-bit index arithmetic: the image is ~0.5 M floats, and 64-bit divisions dominated the pack)
__device__ __forceinline__ void pack_fp32_at(const RawParams& rp, float* __restrict__ out, const int64_t idx64) {
  if (idx64 >= kPackedFloats) return;
  static_assert(kPackedFloats < (1LL << 31), "32-bit pack indices");
  const int idx = (int)idx64;
  float v = 0.f;
  auto frag = [](int i, int& kc, int& t, int& r, int& lane, int tiles) {
    // [kc][t][rq][lane][4]
    const int per_chunk = tiles * 1024;
    kc = i / per_chunk;
    int rem = i % per_chunk;
    t = rem >> 10;
    rem &= 1023;
    const int rq = rem >> 8;
    lane = (rem & 255) >> 2;
    r = rq * 4 + (rem & 3);
  };
  int kc, t, r, lane;
  if (idx < kOffOF) {  // forward hidden images
    int layer, i;
    if (idx < kOffL1F) { layer = 0; i = idx - (int)kOffL0F; }
    else if (idx < kOffL2F) { layer = 1; i = idx - (int)kOffL1F; }
    else if (idx < kOffL3F) { layer = 2; i = idx - (int)kOffL2F; }
    else { layer = 3; i = idx - (int)kOffL3F; }
    frag(i, kc, t, r, lane, 8);
    const int row = 32 * t + (lane & 31);
    const int col = 32 * kc + perm(r, lane >> 5);
    const float* W = rp.at(1 + 2 * layer);
    if (layer == 0) v = col < kFourier ? W[row * kFourier + col] : 0.f;
    else v = W[row * kHidden + col];
  } else if (idx < kOffB0) {  // output layer forward image [kc][rq][lane][4]
    frag(idx - (int)kOffOF, kc, t, r, lane, 1);
    const int row = lane & 31;
    const int col = 32 * kc + perm(r, lane >> 5);
    v = row < 4 ? rp.p[9][row * kHidden + col] : 0.f;
  } else if (idx < kOffBO) {  // bias images [t][rq][lane][4]
    const int layer = (idx - (int)kOffB0) / (int)kBiasFloats;
    frag((idx - (int)kOffB0) % (int)kBiasFloats, kc, t, r, lane, 8);
    v = rp.at(2 + 2 * layer)[32 * t + perm(r, lane >> 5)];
  } else if (idx < kOffFB) {  // output bias [rq][lane][4]
    frag(idx - (int)kOffBO, kc, t, r, lane, 1);
    const int u = perm(r, lane >> 5);
    v = u < 4 ? rp.p[10][u] : 0.f;
  } else if (idx < kOffOT) {  // Fourier B padded [3][96]
    const int i = (int)(idx - kOffFB);
    const int c = i / kFourierPad, k = i % kFourierPad;
    v = k < kFourier ? rp.p[0][c * kFourier + k] : 0.f;
  } else if (idx < kOffL3T) {  // Wo^T [t][lane][4]: k-steps r = 0..3 only
    const int i = (int)(idx - kOffOT);
    t = i / 256;
    lane = (i % 256) / 4;
    r = i % 4;
    const int o = perm(r, lane >> 5);
    v = o < 4 ? rp.p[9][o * kHidden + 32 * t + (lane & 31)] : 0.f;
  } else if (idx < kOffL0T) {  // W_l^T, l = 3,2,1
    const int which = (idx - (int)kOffL3T) / (int)(8 * kChunkFloats);  // 0:W3 1:W2 2:W1
    frag((idx - (int)kOffL3T) % (int)(8 * kChunkFloats), kc, t, r, lane, 8);
    const float* W = rp.at(7 - 2 * which);
    const int row = 32 * t + (lane & 31);         // input unit of W
    const int col = 32 * kc + perm(r, lane >> 5);  // output unit of W (the K index here)
    v = W[col * kHidden + row];
  } else {  // W0^T, 3 out tiles
    frag(idx - (int)kOffL0T, kc, t, r, lane, 3);
    const int row = 32 * t + (lane & 31);
    const int col = 32 * kc + perm(r, lane >> 5);
    v = row < kFourier ? rp.p[1][col * kFourier + row] : 0.f;
  }
  out[idx] = v;
}

// fc_c fp32 image element idx (pnr_internal.h "fc_c image"): fc[2l] = fc_c.l.weight (256,32),
// fc[2l+1] = bias; segments 0..3 CF_l, 4..7 CB_l, 8..11 CT (reversed)
struct FcRaw {
  const float* p[PNR_N_FC_PARAMS];
};
__device__ __forceinline__ void fc_pack_fp32_at(const FcRaw& fc, float* __restrict__ out, int64_t idx) {
  if (idx >= kFcPackedFloats) return;
  const int seg = (int)(idx / kChunkFloats);
  const int i = (int)(idx % kChunkFloats);
  const int blk = i / 1024, rem = i % 1024;   // blk = tile t (CF, CB) or k-chunk kc (CT)
  const int rq = rem / 256, lane = (rem % 256) / 4, r = rq * 4 + rem % 4;
  const int hh = lane >> 5, i32 = lane & 31;
  float v;
  if (seg < 4) {
    v = fc.p[2 * seg][(32 * blk + i32) * kCDim + perm(r, hh)];
  } else if (seg < 8) {
    v = fc.p[2 * (seg - 4) + 1][32 * blk + perm(r, hh)];
  } else {
    const int l = 3 - (seg - 8);  // the backward visits l = 3, 2, 1, 0
    v = fc.p[2 * l][(32 * blk + perm(r, hh)) * kCDim + i32];
  }
  out[idx] = v;
}

}  // namespace pnr
