// tr_mnl.h — host/device interface of the factored single-pass multinomial kernel
// (multinomial_tensor_regression.py: model 148-187, the CrossEntropyLoss of fit_Adam 448-457).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace tr {

constexpr int kMnlRMax = 32;  // rank bound of the factored kernel (8 rank blocks of 4)
constexpr int kMnlCMax = 16;  // classes: one 16-lane DPP row
constexpr int kMnlGMax = 8;   // LDS-DMA instructions per wave per sample (sample <= 64 KiB)

// Geometry of one multinomial model with two feature modes, X (N, I, J), factors
// Phi0 (I x R), Phi1 (J x R), PhiC (C x R), passed to the kernel by value.
//
// Per sample the kernel never forms the dense (I*J x C) coefficient tensor: it contracts X_n
// with the two feature factors directly,
//     T[i, r] = sum_j X_n[i, j] Phi1[j, r]      (A-units)
//     V[j, r] = sum_i X_n[i, j] Phi0[i, r]      (B-units)
// on v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4 outer products: 4 ranks per instruction, no
// padding of R to 16).  A unit is a (64 output rows) x (64-deep k range) x (4 ranks) tile of
// one of the two GEMMs; each wave owns upw <= 2 units and keeps their B operands (64 factor
// values per lane) in registers for the whole launch.
struct MnlGeom {
  int I, J, R, C;
  int JQ;         // 16-B chunks per X row (J / 4)
  int smask;      // XOR swizzle of the chunk index in LDS (row i: chunk q stored at q ^ (i & smask))
  int nchunk;     // 16-B chunks per sample (I * J / 4)
  int nbuf;       // LDS ring depth (samples)
  int nib, njb, nrb, Rp;  // 64-row blocks of I and J, rank blocks of 4, Rp = 4 * nrb
  int nA, nunits, upw, nsets;  // A-units, all units (2 nA, one per wave), units per wave (1), nib * njb
  int full;       // I % 64 == 0 && J % 64 == 0 (no k-range guards)
  int spi;        // samples per barrier (2 when the ring holds >= 2 pairs)
  int64_t offP1, offPC, nfelem, slab;  // arena offsets (floats); slab stride (nfelem rounded to 4)
  // LDS carve (floats)
  int oZ, oG, lds_floats;  // oZ: [2][2][16][4] Z partials; oG: LDS image of the arena (aliases the drained ring)
  // two-workgroups-per-CU variant (tr_mnl_duo.hip): 4 waves, each owning every rank block of
  // one (i, j) block; LDS carve of ONE workgroup (floats)
  int duo;
  int du_oZ, du_oP1, du_oG, du_lds_floats;
  // bf16-split form of the duo family (k_mnl_bsp: a 32 KiB (128, 64) or (64, 128) sample at
  // rank <= 4, and every (32 NW, 64) sample with NW = 2..8 and (16 NW, 128) sample with NW = 4, 6,
  // 8 at rank <= 8 (other I, and J % 4 == 0 of 28..128, padded to the next; taller samples as du_nb
  // row blocks of those), C <= 16; TR_DUO_SPLIT=1
  // takes it at (128, 64) / (64, 128) rank 5..8 too, =0 keeps the rank-block form): U partials at bs_oU
  int bsp, bs_oU;
  // split body's X form (tr_plan_set_x_range): 0 = bf16 + f16 residual, 1 = three exact bf16 pieces
  int bs_exact;
  // waves per workgroup and workgroups per CU of the two-workgroups-per-CU family (4, 2; the
  // split body on (32 NW, 64) and (16 NW, 128) samples: NW, 8 / NW)
  int du_nw, du_wpc;
  int du_ns;  // split body: samples in the LDS ring (2; 3 at NW = 5, 6)
  int du_pad;  // split body: g.I x g.J fills only part of the compiled (32 NW or 16 NW) x du_jt sample
  int du_jt;   // the duo family's compiled row width (J, or 64 / 128 above a padded J)
  // split body's row blocks per sample (1; a sample of du_nb * 32 NW (J <= 64) or du_nb * 16 NW rows
  // streams through the ring one row block per slot) and the LDS offset of the earlier blocks' T / dPhi0
  int du_nb, bs_oTB;
  int bs_oW;  // bsp: [ns][8] published Wv of the one-wave epilogue (J = 32), then [8] per-wave loss partials (double)
  // split body's rank columns: 8 (R <= 8: two pieces of 8 ranks per 16-column tile, folded) or 16
  // (R 9..16: 16 ranks of one piece per tile)
  int bs_rk;
  // k_mnl_fused fits this shape (mnl_geom_init may accept a shape only the split body runs)
  int fused_ok;
};

// Fills g; false (with a reason) when the shape is outside the factored kernels' envelope.  A
// shape k_mnl_fused does not fit (more than 8 GEMM units, its LDS ring) returns true with
// g->fused_ok = 0 (and the reason): only the split body of tr_mnl_duo.hip can run it.
bool mnl_geom_init(MnlGeom* g, int64_t I, int64_t J, int R, int C, std::string* why);
// Sets the dynamic-LDS limit and checks the instantiation is spill-free and fits a CU.
hipError_t mnl_prepare(const MnlGeom& g, int* ok);
// One workgroup per CU over a contiguous sample range (reversed when `reverse`).  Writes one
// phi-space gradient slab per workgroup in arena layout [dPhi0 | dPhi1 | dPhiC] (stride g.slab)
// and (sum_n cw[y_n] * CE_n, 0) into dpart[2 * wg].
hipError_t launch_mnl_fused(const MnlGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                            const float* w, const int64_t* lab, const float* class_w, float scale, float* gpart,
                            double* dpart, int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st);

// Two-workgroups-per-CU variant (tr_mnl_duo.hip): sets g->duo when the shape fits it (two 64-row
// blocks, R <= 8, LDS for two workgroups; TR_MNL_DUO=0 turns it off), then checks the compiled
// kernel is spill-free and two of its workgroups fit a CU.
void mnl_duo_geom(MnlGeom* g);
hipError_t mnl_duo_prepare(MnlGeom* g);
// Same contract as launch_mnl_fused, with grid = g.du_wpc workgroups per CU.
hipError_t launch_mnl_duo(const MnlGeom& g, int grid, const float* X, int64_t N, int64_t xld, const float* phi,
                          const float* w, const int64_t* lab, const float* class_w, float scale, float* gpart,
                          double* dpart, int64_t rows_per_wg, int reverse, const int32_t* stop, hipStream_t st);

}  // namespace tr
