// tr_api.hip — the C ABI (include/tensor_regression_hip.h): plans, workspace, kernel strategy.
//
// A plan is the MI355X-side image of one CP_linear_regression / CP_logistic_regression shape
// (standard_tensor_regression.py:204-303, multinomial_tensor_regression.py:212-286): the
// Kruskal factor layout, the dense-coefficient workspace and the per-iteration scratch.
// All device buffers the caller passes in are borrowed; the plan owns only its workspace.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tensor_regression_hip.h"
#include "tr_kernels.h"
#include "tr_mnl.h"
#include "tr_spectral.h"

using namespace tr;

struct tr_plan {
  int device = 0;
  int model = TR_MODEL_LINEAR;
  int K = 0;  // feature modes
  int C = 1;  // classes (1 for linear)
  int R = 0;
  int has_bias = 1;
  float sp_beta = 50.f, sp_thr = 1.f;
  int64_t P = 0, ncols = 0, nparams = 0, ngrads = 0, max_rows = 0;
  int64_t xld = 0;  // row stride of X in floats (P unless tr_plan_set_x_stride)
  FactorSet fs{};
  int ncu = 256;
  int W = 4;
  // single-pass linear strategy
  int fused = 0, fT = 0, fCH = 0, fgrid = 0;
  int mfma_rows = 0;  // multinomial forward on the matrix cores
  // single-pass linear strategy for P beyond one CU's LDS (clusters of cS workgroups)
  int cluster = 0, cCH = 0, cS = 0, cncl = 0;
  unsigned long long* gran = nullptr;  // cluster exchange granules (2 row slots x S per cluster)
  uint32_t* err_word = nullptr;        // device status word (bit 0: a cluster exchange timed out)
  uint32_t cl_tag = 0;                 // last granule tag used (tags only grow; wrap -> re-zero)
  int64_t gran_n = 0;
  // single-pass factored multinomial strategy (two feature modes, tr_mnl.hip)
  int mnl = 0;
  MnlGeom mg{};
  // spectral model (TR_MODEL_SPECTRAL)
  SpecGeom sg{};
  float* Phi0 = nullptr;
  int sgrid = 0;
  int64_t slab_stride = 0;
  // two-pass strategy
  int64_t max_slabs = 0;
  // next-iteration factor preparation folded into tr_adam_step (tr_plan_set_prepare_next)
  int prep_next = 0;
  int prepared = 0;  // 1: phi / dphi hold the factors of prep_params
  const float* prep_params = nullptr;
  // workspace
  void* ws = nullptr;
  size_t ws_bytes = 0;
  float *phi = nullptr, *dphi = nullptr, *dense = nullptr, *G = nullptr, *gpart = nullptr, *rowbuf = nullptr;
  double* dpart = nullptr;
  int64_t gpart_slabs = 0, dpart_n = 0;
  unsigned parity = 0;
  std::string desc;
  // optional per-kernel event timing (tr_plan_set_timing)
  int timing = 0;  // bit mask of timed TR_KERNEL_* kinds
  struct Rec {
    hipEvent_t a, b;
    int kind;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
};

static hipEvent_t take_event(tr_plan* p) {
  if (!p->pool.empty()) {
    hipEvent_t e = p->pool.back();
    p->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one kernel launch with events when timing is on (no host synchronisation).
struct TimedLaunch {
  tr_plan* p;
  hipStream_t st;
  int kind;
  hipEvent_t a = nullptr;
  TimedLaunch(tr_plan* p_, hipStream_t st_, int kind_) : p(p_), st(st_), kind(kind_) {
    if (p->timing & (1 << kind)) {
      a = take_event(p);
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~TimedLaunch() {
    if (a) {
      hipEvent_t b = take_event(p);
      if (b) {
        (void)hipEventRecord(b, st);
        p->recs.push_back({a, b, kind});
      } else {
        p->pool.push_back(a);
      }
    }
  }
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
static int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return (int)e;
}
#define TR_HIP(expr)                                   \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return hip_fail(_e, #expr);  \
  } while (0)

static bool env_flag(const char* name) {
  const char* v = std::getenv(name);
  return v != nullptr && v[0] != '\0' && v[0] != '0';
}

extern "C" int tr_abi_version(void) { return TR_ABI_VERSION; }
extern "C" const char* tr_last_error(void) { return g_err.c_str(); }

// Single-pass strategy for the linear model: among the (T, CH) with P == 4*T*CH, keep the
// spill-free instantiations and pick the one with the most X bytes in flight per CU (one
// prefetched row per resident workgroup), ties to the smaller workgroup.
static void choose_fused(tr_plan* p) {
  p->fused = 0;
  if (p->model != TR_MODEL_LINEAR || p->P % 4 != 0 || p->xld % 4 != 0 || env_flag("TR_FORCE_TWOPASS")) return;
  const int64_t P4 = p->P / 4;
  const size_t lds_max = 160 * 1024;
  const int Ts[5] = {64, 128, 256, 512, 1024};
  int64_t best_bytes = 0;
  int best_waves = 1 << 30;
  const char* force_t = std::getenv("TR_FUSED_T");  // experiment knob
  for (int k = 0; k < 5; ++k) {
    const int T = Ts[k];
    if (force_t != nullptr && std::atoi(force_t) != T) continue;
    if (P4 % T != 0) continue;
    const int64_t CH = P4 / T;
    if (!linear_fused_supported(T, (int)CH)) continue;
    const size_t lds = (size_t)p->P * 4 + 2 * (T / 64) * 4;
    if (lds > lds_max) continue;
    int per_cu = 0;
    if (prepare_linear_fused(T, (int)CH, lds, &per_cu) != hipSuccess || per_cu < 1) continue;
    const int64_t bytes = (int64_t)per_cu * p->P * 4;
    const int waves = per_cu * T / 64;
    // most X bytes in flight per CU; ties -> fewer waves per barrier (with nt loads the
    // config-2 row streams at 6.80 TB/s with T=512 vs 6.70 with T=1024)
    if (bytes > best_bytes || (bytes == best_bytes && waves < best_waves)) {
      best_bytes = bytes;
      best_waves = waves;
      p->fused = 1;
      p->fT = T;
      p->fCH = (int)CH;
      p->fgrid = p->ncu * per_cu;
    }
  }
}

// Single pass for a linear P too wide for one CU's LDS: clusters of S workgroups split every row
// into S feature slices (tr_cluster.hip).  Among the spill-free slice widths pick the one that
// wastes the fewest lanes: P / (S * slice) for the padding of the last slice, times the
// fraction of CUs the floor(ncu / S) clusters keep busy.
static void choose_cluster(tr_plan* p) {
  p->cluster = 0;
  if (p->model != TR_MODEL_LINEAR || p->fused || p->P % 4 != 0 || p->xld % 4 != 0 || env_flag("TR_FORCE_TWOPASS") ||
      env_flag("TR_NO_CLUSTER"))
    return;
  const char* force_ch = std::getenv("TR_CLUSTER_CH");  // experiment knob
  double best = 0.0;
  for (int k = 0; k < linear_cluster_num_ch(); ++k) {
    const int CH = linear_cluster_ch(k);
    if (force_ch != nullptr && std::atoi(force_ch) != CH) continue;
    const int64_t PS = linear_cluster_slice(CH);
    const int64_t S = (p->P + PS - 1) / PS;
    if (S < 2 || S > 64 || S > p->ncu) continue;
    int per_cu = 0;
    if (prepare_linear_cluster(CH, &per_cu) != hipSuccess || per_cu < 1) continue;
    const int64_t ncl = p->ncu / S;  // one workgroup per CU: every member co-resident
    const double score = (double)p->P / (double)(S * PS) * (double)(ncl * S) / (double)p->ncu;
    if (score > best + 1e-9) {
      best = score;
      p->cluster = 1;
      p->cCH = CH;
      p->cS = (int)S;
      p->cncl = (int)ncl;
    }
  }
}

// Single pass for the multinomial model with two feature modes: the factored kernel contracts X
// with Phi0 / Phi1 directly (no dense B) and reads every X row once (tr_mnl.hip).
static void choose_mnl(tr_plan* p) {
  p->mnl = 0;
  if (p->model != TR_MODEL_MULTINOMIAL || p->K != 2 || p->xld % 4 != 0 || env_flag("TR_FORCE_TWOPASS") ||
      env_flag("TR_NO_MNL_FUSED"))
    return;
  MnlGeom g;
  if (!mnl_geom_init(&g, p->fs.dim[0], p->fs.dim[1], p->R, p->C, nullptr)) return;
  int ok = 0;
  if (mnl_prepare(g, &ok) != hipSuccess || !ok) return;
  p->mg = g;
  p->mnl = 1;
}

extern "C" int tr_plan_create(tr_plan** out, int device, int model, int n_feature_modes,
                              const int64_t* feature_dims, int n_classes, int rank, int64_t max_rows,
                              const int32_t* non_negative, float softplus_beta,
                              float softplus_threshold) {
  if (out == nullptr) return fail(TR_E_ARG, "out is NULL");
  *out = nullptr;
  if (model != TR_MODEL_LINEAR && model != TR_MODEL_MULTINOMIAL) return fail(TR_E_ARG, "unknown model");
  const int nf = n_feature_modes + (model == TR_MODEL_MULTINOMIAL ? 1 : 0);
  if (n_feature_modes < 1 || nf > TR_MAXF) return fail(TR_E_ARG, "number of factors out of range [1, 8]");
  if (rank < 1 || rank > TR_MAXR) return fail(TR_E_ARG, "rank out of range [1, 64]");
  if (feature_dims == nullptr) return fail(TR_E_ARG, "feature_dims is NULL");
  if (max_rows < 1) return fail(TR_E_ARG, "max_rows must be >= 1");
  const int C = model == TR_MODEL_MULTINOMIAL ? n_classes : 1;
  if (C < 1) return fail(TR_E_ARG, "n_classes must be >= 1");
  if (!rows_supported(C)) return fail(TR_E_UNSUPPORTED, "n_classes > 16 not supported by the gfx950 kernels yet");

  tr_plan* p = new tr_plan();
  p->device = device;
  p->model = model;
  p->K = n_feature_modes;
  p->C = C;
  p->R = rank;
  p->has_bias = model == TR_MODEL_LINEAR;
  p->sp_beta = softplus_beta;
  p->sp_thr = softplus_threshold;
  p->max_rows = max_rows;

  int64_t P = 1;
  for (int k = 0; k < n_feature_modes; ++k) {
    if (feature_dims[k] < 1) {
      delete p;
      return fail(TR_E_ARG, "feature dims must be >= 1");
    }
    P *= feature_dims[k];
  }
  p->P = P;
  p->xld = P;
  p->ncols = P * C;
  if (p->ncols >= ((int64_t)1 << 31)) {
    delete p;
    return fail(TR_E_UNSUPPORTED, "prod(dims) * n_classes must be < 2^31");
  }
  FactorSet& fs = p->fs;
  std::memset(&fs, 0, sizeof(fs));
  fs.nf = nf;
  fs.rank = rank;
  for (int f = 0; f < nf; ++f) {
    fs.dim[f] = f < n_feature_modes ? feature_dims[f] : C;
    fs.nonneg[f] = non_negative ? (non_negative[f] != 0) : 0;
  }
  int64_t off = 0, rs = 1;
  for (int f = 0; f < nf; ++f) {
    fs.off[f] = off;
    off += fs.dim[f] * rank;
  }
  for (int f = nf - 1; f >= 0; --f) {
    fs.rstride[f] = rs;
    rs *= fs.dim[f];
  }
  fs.total = rs;
  fs.nfelem = off;
  // dense layout: row-major over feature modes; class factor (multinomial) slowest
  int64_t ds = 1;
  for (int f = n_feature_modes - 1; f >= 0; --f) {
    fs.stride[f] = ds;
    ds *= fs.dim[f];
  }
  if (model == TR_MODEL_MULTINOMIAL) fs.stride[n_feature_modes] = P;
  for (int f = 0; f < nf; ++f) {  // other factors of f by decreasing dense stride (MTTKRP walk order)
    int k = 0;
    for (int g = 0; g < nf; ++g)
      if (g != f) fs.others[f][k++] = (int8_t)g;
    for (int a = 1; a < k; ++a)
      for (int b = a; b > 0 && fs.stride[fs.others[f][b - 1]] < fs.stride[fs.others[f][b]]; --b) {
        const int8_t t = fs.others[f][b];
        fs.others[f][b] = fs.others[f][b - 1];
        fs.others[f][b - 1] = t;
      }
  }
  p->nparams = fs.nfelem + (p->has_bias ? 1 : 0);
  p->ngrads = p->nparams + 1;
  p->W = (P % 4 == 0) ? 4 : 1;

  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipSetDevice");
  }
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    p->ncu = ncu;

  choose_fused(p);
  choose_cluster(p);
  choose_mnl(p);
  p->mfma_rows = (model == TR_MODEL_MULTINOMIAL && rows_mfma_supported(C, P) && !env_flag("TR_NO_MFMA")) ? 1 : 0;

  // two-pass slab budget: max(16 MiB, 2 % of X bytes)
  {
    const double xbytes = (double)max_rows * (double)P * 4.0;
    double budget = xbytes * 0.02;
    if (budget < 16.0 * 1024 * 1024) budget = 16.0 * 1024 * 1024;
    int64_t ms = (int64_t)(budget / ((double)p->ncols * 4.0));
    if (ms < 1) ms = 1;
    if (ms > 1024) ms = 1024;
    p->max_slabs = ms;
  }
  p->gpart_slabs = p->max_slabs;
  if (p->fused && p->fgrid > p->gpart_slabs) p->gpart_slabs = p->fgrid;
  p->dpart_n = rows_num_waves(C, max_rows) + rows_mfma_num_waves(max_rows) + 64;
  if (p->fused && p->fgrid > p->dpart_n) p->dpart_n = p->fgrid;
  if (p->cluster && p->cncl > p->gpart_slabs) p->gpart_slabs = p->cncl;
  if (p->cluster && p->cncl > p->dpart_n) p->dpart_n = p->cncl;
  if (p->mnl && p->ncu > p->dpart_n) p->dpart_n = p->ncu;
  p->gran_n = 2 * (int64_t)p->ncu;  // >= 2 slots x S x ncl for any cluster shape

  // workspace carve (256-B aligned pieces)
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  // dense B / G: class-major; padded to 16 class rows for the MFMA forward (pad rows stay zero)
  const int64_t dense_rows = p->mfma_rows && C < 16 ? 16 : C;
  size_t b_gpart = al((size_t)p->gpart_slabs * p->ncols * 4), b_dense = al((size_t)dense_rows * P * 4);
  if (p->mnl) {  // one arena-layout slab per CU; G holds the reduced arena
    if (b_gpart < al((size_t)p->ncu * p->mg.slab * 4)) b_gpart = al((size_t)p->ncu * p->mg.slab * 4);
    if (b_dense < al((size_t)p->mg.slab * 4)) b_dense = al((size_t)p->mg.slab * 4);
  }
  const size_t b_phi = al(fs.nfelem * 4),
               b_row = al((size_t)max_rows * C * 4), b_dpart = al((size_t)p->dpart_n * 2 * 8),
               b_gran = al((size_t)p->gran_n * 8 + 16);
  p->ws_bytes = 2 * b_phi + 2 * b_dense + b_gpart + b_row + b_dpart + b_gran;
  e = hipMalloc(&p->ws, p->ws_bytes);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipMalloc(workspace)");
  }
  char* c = (char*)p->ws;
  p->phi = (float*)c;
  c += b_phi;
  p->dphi = (float*)c;
  c += b_phi;
  p->dense = (float*)c;
  c += b_dense;
  p->G = (float*)c;
  c += b_dense;
  p->gpart = (float*)c;
  c += b_gpart;
  p->rowbuf = (float*)c;
  c += b_row;
  p->dpart = (double*)c;
  c += b_dpart;
  p->gran = (unsigned long long*)c;
  p->err_word = (uint32_t*)(c + p->gran_n * 8);
  TR_HIP(hipMemset(p->ws, 0, p->ws_bytes));

  char buf[512];
  std::snprintf(buf, sizeof(buf),
                "model=%s K=%d C=%d R=%d P=%lld nparams=%lld ncu=%d path=%s%s T=%d CH=%d grid=%d W=%d "
                "max_slabs=%lld workspace=%.1fMiB",
                model == TR_MODEL_LINEAR ? "linear" : "multinomial", p->K, C, rank, (long long)P,
                (long long)p->nparams, p->ncu,
                p->fused ? "fused-1pass" : (p->cluster ? "cluster-1pass" : (p->mnl ? "mnl-fused-1pass" : "2pass")),
                p->mfma_rows ? "+mfma-fwd" : "", p->cluster ? 512 : p->fT, p->cluster ? p->cCH : p->fCH,
                p->cluster ? p->cS * p->cncl : p->fgrid, p->W, (long long)p->max_slabs, p->ws_bytes / 1048576.0);
  if (p->cluster) {
    char b2[96];
    std::snprintf(b2, sizeof(b2), " S=%d clusters=%d", p->cS, p->cncl);
    std::strncat(buf, b2, sizeof(buf) - std::strlen(buf) - 1);
  }
  if (p->mnl) {
    char b2[128];
    std::snprintf(b2, sizeof(b2), " units=%d nbuf=%d lds=%.1fKiB", p->mg.nunits, p->mg.nbuf,
                  p->mg.lds_floats * 4 / 1024.0);
    std::strncat(buf, b2, sizeof(buf) - std::strlen(buf) - 1);
  }
  p->desc = buf;
  *out = p;
  return 0;
}

// Spectral plan (spectral_tensor_regression.CP_linear_regression.__init__, :425-539): the
// parameter arena is Bcp_n + Bcp_c + [bias] in the reference's order; the per-iteration
// pipeline is prep -> fused single pass -> slab reduction -> softplus chain.
extern "C" int tr_plan_create_spectral(tr_plan** out, int device, int64_t n_w, int64_t n_d, int64_t n_out,
                                       int rank_normal, int rank_spectral, int n_complex, int64_t max_rows,
                                       const int32_t* non_negative, float softplus_beta,
                                       float softplus_threshold) {
  if (out == nullptr) return fail(TR_E_ARG, "out is NULL");
  *out = nullptr;
  if (max_rows < 1) return fail(TR_E_ARG, "max_rows must be >= 1");
  if (n_w < 1 || n_d < 1 || n_out < 1 || rank_normal < 0 || rank_spectral < 0 || n_complex < 1)
    return fail(TR_E_ARG, "spectral dims / ranks out of range");
  if (rank_normal + rank_spectral < 1) return fail(TR_E_ARG, "rank_normal + rank_spectral must be >= 1");
  tr_plan* p = new tr_plan();
  std::string why;
  if (!spec_geom_init(&p->sg, n_w, n_d, n_out, rank_normal, rank_spectral, n_complex, non_negative, &why)) {
    delete p;
    return fail(TR_E_UNSUPPORTED, why);
  }
  const SpecGeom& g = p->sg;
  p->device = device;
  p->model = TR_MODEL_SPECTRAL;
  p->K = 2;
  p->C = (int)n_out;
  p->R = rank_normal + rank_spectral;
  p->has_bias = (int)n_out;  // bias entries (one per output)
  p->sp_beta = softplus_beta;
  p->sp_thr = softplus_threshold;
  p->max_rows = max_rows;
  p->P = g.WD;
  p->xld = g.WD;
  p->nparams = g.nparams;
  p->ngrads = g.nparams + 1;
  FactorSet& fs = p->fs;
  std::memset(&fs, 0, sizeof(fs));
  fs.nf = 6;
  fs.rank = 0;
  const int64_t offs[6] = {g.offA0, g.offA1, g.offA2, g.offC0, g.offC1, g.offC2};
  const int64_t dims[6] = {n_w, n_d, n_out, n_w, n_d, n_out};
  for (int f = 0; f < 6; ++f) {
    fs.off[f] = offs[f];
    fs.dim[f] = dims[f];
    fs.nonneg[f] = g.nonneg[f % 3];
  }
  fs.nfelem = g.offB;
  fs.total = 0;

  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipSetDevice");
  }
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    p->ncu = ncu;
  for (int mode = SPEC_TRAIN; mode <= SPEC_LATENT; ++mode) {
    int ok = 0;
    e = spec_prepare(g, mode, &ok);
    if (e != hipSuccess) {
      delete p;
      return hip_fail(e, "spec_prepare");
    }
    if (!ok) {
      delete p;
      return fail(TR_E_UNSUPPORTED, "spectral kernel does not fit a CU for this shape");
    }
  }
  p->sgrid = p->ncu;  // one workgroup per CU (the kernel holds one sample in 150 KiB of LDS)
  p->slab_stride = (g.nparams + 3) & ~(int64_t)3;
  p->gpart_slabs = p->sgrid;
  p->dpart_n = p->sgrid;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_par = al((size_t)g.nparams * 4), b_phi0 = al((size_t)g.W * g.K * 4),
               b_G = al((size_t)p->slab_stride * 4), b_gpart = al((size_t)p->sgrid * p->slab_stride * 4),
               b_dpart = al((size_t)p->dpart_n * 2 * 8);
  p->ws_bytes = 2 * b_par + b_phi0 + b_G + b_gpart + b_dpart;
  e = hipMalloc(&p->ws, p->ws_bytes);
  if (e != hipSuccess) {
    delete p;
    return hip_fail(e, "hipMalloc(workspace)");
  }
  char* c = (char*)p->ws;
  p->phi = (float*)c;
  c += b_par;
  p->dphi = (float*)c;
  c += b_par;
  p->Phi0 = (float*)c;
  c += b_phi0;
  p->G = (float*)c;
  c += b_G;
  p->gpart = (float*)c;
  c += b_gpart;
  p->dpart = (double*)c;
  TR_HIP(hipMemset(p->ws, 0, p->ws_bytes));
  char buf[512];
  std::snprintf(buf, sizeof(buf),
                "model=spectral W=%d D=%d n_out=%d Rn=%d Rs=%d Cc=%d K=%d nparams=%lld ncu=%d path=fused-1pass-mfma "
                "KT=%d S=%d grid=%d lds=%.1fKiB vec=%d workspace=%.1fMiB",
                g.W, g.D, g.NO, g.Rn, g.Rs, g.Cc, g.K, (long long)g.nparams, p->ncu, g.KT, g.S, p->sgrid,
                g.lds_floats * 4 / 1024.0, g.vec, p->ws_bytes / 1048576.0);
  p->desc = buf;
  *out = p;
  return 0;
}

// Row stride of X (strided / windowed views: row n starts at X + n*stride, its P floats
// contiguous).  Vector (16-B) kernel paths need stride % 4 == 0 and a 16-B aligned X.
extern "C" int tr_plan_set_x_stride(tr_plan* p, int64_t stride) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (stride < 0) return fail(TR_E_ARG, "stride must be >= 0 (0 = dense rows)");
  const int64_t x = stride == 0 ? p->P : stride;
  p->xld = x;
  if (p->model == TR_MODEL_SPECTRAL) {
    p->sg.vec = (p->sg.WD % 4 == 0 && x % 4 == 0) ? 1 : 0;
    return 0;
  }
  TR_HIP(hipSetDevice(p->device));
  p->W = (p->P % 4 == 0 && x % 4 == 0) ? 4 : 1;
  const int had_fused = p->fused;
  const int64_t fgrid = p->fgrid;
  choose_fused(p);
  if (p->fused && (!had_fused || p->fgrid > fgrid)) {
    // the workspace was carved for the creation-time strategy; keep within it
    p->fused = had_fused;
    p->fgrid = fgrid;
  }
  const int had_cluster = p->cluster;
  const int cncl = p->cncl;
  choose_cluster(p);
  if (p->cluster && (!had_cluster || p->cncl > cncl)) p->cluster = 0;  // keep within the workspace
  const int had_mnl = p->mnl;
  choose_mnl(p);
  if (p->mnl && !had_mnl) p->mnl = 0;  // keep within the workspace
  p->mfma_rows = (p->model == TR_MODEL_MULTINOMIAL && rows_mfma_supported(p->C, p->P) && x % 4 == 0 &&
                  !env_flag("TR_NO_MFMA"))
                     ? 1
                     : 0;
  return 0;
}

static bool x_vec_paths(const tr_plan* p) {
  if (p->model == TR_MODEL_SPECTRAL) return p->sg.vec != 0;
  return p->W == 4 || p->fused || p->mfma_rows || p->mnl;
}
static int check_x_align(const tr_plan* p, const float* X) {
  if (X != nullptr && x_vec_paths(p) && (reinterpret_cast<uintptr_t>(X) & 15u) != 0)
    return fail(TR_E_ARG, "X must be 16-byte aligned for this plan's vector kernels (or set a stride % 4 != 0)");
  return 0;
}

extern "C" int tr_plan_destroy(tr_plan* p) {
  if (p == nullptr) return 0;
  (void)hipSetDevice(p->device);
  for (auto& r : p->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : p->pool) (void)hipEventDestroy(e);
  if (p->ws) (void)hipFree(p->ws);
  delete p;
  return 0;
}

extern "C" int64_t tr_plan_num_params(const tr_plan* p) { return p ? p->nparams : -1; }
extern "C" int64_t tr_plan_num_grads(const tr_plan* p) { return p ? p->ngrads : -1; }
extern "C" int64_t tr_plan_factor_offset(const tr_plan* p, int f) {
  if (p == nullptr || f < 0 || f > p->fs.nf) return -1;
  return f == p->fs.nf ? p->fs.nfelem : p->fs.off[f];
}
extern "C" int64_t tr_plan_workspace_bytes(const tr_plan* p) { return p ? (int64_t)p->ws_bytes : -1; }
extern "C" const char* tr_plan_describe(const tr_plan* p) { return p ? p->desc.c_str() : ""; }

static int factor_prep(tr_plan* p, const float* params, const float* w, const int32_t* stop, hipStream_t st) {
  p->prepared = 0;
  TimedLaunch tl(p, st, TR_KERNEL_PREP);
  TR_HIP(launch_build_dense(p->fs, params, p->sp_beta, p->sp_thr, p->phi, p->dphi, w, p->dense, stop, st));
  return 0;
}

static int spectral_forward(tr_plan* p, int mode, const float* X, int64_t n_rows, const float* params,
                            const float* weights, float* out, hipStream_t st) {
  {
    TimedLaunch tl(p, st, TR_KERNEL_PREP);
    TR_HIP(launch_spec_prep(p->sg, params, p->sp_beta, p->sp_thr, p->phi, p->dphi, p->Phi0, nullptr, st));
  }
  const int64_t rpw = (n_rows + p->sgrid - 1) / p->sgrid;
  TimedLaunch tl(p, st, TR_KERNEL_STREAM_FUSED);
  TR_HIP(launch_spec_fused(mode, p->sg, p->sgrid, X, n_rows, p->xld, p->phi, p->Phi0, weights, nullptr, 0.f, nullptr, 0,
                           nullptr, out, rpw, 0, nullptr, st));
  return 0;
}

extern "C" int tr_spectral_latents(tr_plan* p, const float* X, int64_t n_rows, const float* params, float* out,
                                   void* stream) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (p->model != TR_MODEL_SPECTRAL) return fail(TR_E_ARG, "tr_spectral_latents needs a spectral plan");
  if (X == nullptr || params == nullptr || out == nullptr) return fail(TR_E_ARG, "NULL buffer");
  if (n_rows < 1 || p->sg.Rn < 1) return 0;
  if (int rc0 = check_x_align(p, X)) return rc0;
  TR_HIP(hipSetDevice(p->device));
  return spectral_forward(p, SPEC_LATENT, X, n_rows, params, nullptr, out, (hipStream_t)stream);
}

extern "C" int tr_forward(tr_plan* p, const float* X, int64_t n_rows, const float* params, const float* weights,
                          float* out, void* stream) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (X == nullptr || params == nullptr || weights == nullptr || out == nullptr)
    return fail(TR_E_ARG, "NULL buffer");
  if (n_rows < 1) return 0;
  if (int rc0 = check_x_align(p, X)) return rc0;
  hipStream_t st = (hipStream_t)stream;
  TR_HIP(hipSetDevice(p->device));
  if (p->model == TR_MODEL_SPECTRAL) return spectral_forward(p, SPEC_PRED, X, n_rows, params, weights, out, st);
  int rc = factor_prep(p, params, weights, nullptr, st);
  if (rc) return rc;
  const int mode = p->model == TR_MODEL_LINEAR ? MODE_LIN_PRED : MODE_MNL_PRED;
  if (p->mfma_rows) {
    TR_HIP(launch_rows_mfma(MODE_MNL_PRED, X, n_rows, p->P, p->xld, p->dense, p->C, nullptr, nullptr, 0.f, out, nullptr,
                            nullptr, st));
    return 0;
  }
  TR_HIP(launch_rows(p->C, mode, p->W, X, n_rows, p->P, p->xld, p->dense, params + p->fs.nfelem, nullptr, nullptr, 0.f,
                     out, nullptr, nullptr, nullptr, st));
  return 0;
}

// True when the previous tr_adam_step already prepared phi / dphi of exactly these params (the
// factored multinomial pass needs nothing else); the mark is consumed either way.
static bool consume_prepared(tr_plan* p, const float* params) {
  const bool ok = p->prepared && p->prep_params == params;
  p->prepared = 0;
  return ok;
}

extern "C" int tr_plan_set_prepare_next(tr_plan* p, int enable) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  p->prep_next = enable ? 1 : 0;
  p->prepared = 0;
  return 0;
}

extern "C" int tr_loss_grad(tr_plan* p, const float* X, int64_t n_rows, const void* target,
                            const float* class_weight, double norm, const float* params, const float* weights,
                            float* grad_out, float* yhat_out, const int32_t* stop_flag, void* stream) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (params == nullptr || weights == nullptr || grad_out == nullptr) return fail(TR_E_ARG, "NULL buffer");
  if (n_rows > 0 && (X == nullptr || target == nullptr)) return fail(TR_E_ARG, "NULL X / target");
  if (p->model == TR_MODEL_MULTINOMIAL && class_weight == nullptr)
    return fail(TR_E_ARG, "multinomial model needs class_weight");
  if (n_rows < 0 || n_rows > p->max_rows) return fail(TR_E_ARG, "n_rows exceeds the plan's max_rows");
  if (!(norm > 0.0)) return fail(TR_E_ARG, "norm must be > 0");
  if (n_rows > 0)
    if (int rc0 = check_x_align(p, X)) return rc0;
  hipStream_t st = (hipStream_t)stream;
  TR_HIP(hipSetDevice(p->device));
  if (n_rows == 0) {
    // an empty shard contributes nothing to the all-reduced sum
    TR_HIP(hipMemsetAsync(grad_out, 0, (size_t)p->ngrads * 4, st));
    return 0;
  }
  if (p->model == TR_MODEL_SPECTRAL) {
    const int reverse = (int)(p->parity & 1u);
    p->parity++;
    {
      TimedLaunch tl(p, st, TR_KERNEL_PREP);
      TR_HIP(launch_spec_prep(p->sg, params, p->sp_beta, p->sp_thr, p->phi, p->dphi, p->Phi0, stop_flag, st));
    }
    const int64_t rpw = (n_rows + p->sgrid - 1) / p->sgrid;
    {
      TimedLaunch tl(p, st, TR_KERNEL_STREAM_FUSED);
      TR_HIP(launch_spec_fused(SPEC_TRAIN, p->sg, p->sgrid, X, n_rows, p->xld, p->phi, p->Phi0, weights,
                               (const float*)target, (float)(2.0 / norm), p->gpart, p->slab_stride, p->dpart, yhat_out,
                               rpw, reverse, stop_flag, st));
    }
    {
      TimedLaunch tl(p, st, TR_KERNEL_REDUCE);
      TR_HIP(launch_reduce_slabs(4, p->gpart, p->sgrid, p->slab_stride, p->G, p->dpart, p->sgrid, 1.0 / norm,
                                 grad_out + p->nparams, nullptr, stop_flag, st, p->dphi, grad_out, p->nparams));
    }
    return 0;
  }
  if (p->mnl) {
    const int reverse = (int)(p->parity & 1u);
    p->parity++;
    if (!consume_prepared(p, params)) {
      TimedLaunch tl(p, st, TR_KERNEL_PREP);
      TR_HIP(launch_prep_factors(p->fs, params, p->sp_beta, p->sp_thr, p->phi, p->dphi, stop_flag, st));
    }
    const int grid = p->ncu;
    const int64_t rpw = (n_rows + grid - 1) / grid;
    {
      TimedLaunch tl(p, st, TR_KERNEL_STREAM_FUSED);
      TR_HIP(launch_mnl_fused(p->mg, grid, X, n_rows, p->xld, p->phi, weights, (const int64_t*)target, class_weight,
                              (float)(1.0 / norm), p->gpart, p->dpart, rpw, reverse, stop_flag, st));
    }
    {
      TimedLaunch tl(p, st, TR_KERNEL_REDUCE);
      TR_HIP(launch_reduce_slabs(4, p->gpart, grid, p->mg.slab, p->G, p->dpart, grid, 1.0 / norm,
                                 grad_out + p->nparams, nullptr, stop_flag, st, p->dphi, grad_out, p->fs.nfelem));
    }
    return 0;
  }
  p->prepared = 0;
  int rc = factor_prep(p, params, weights, stop_flag, st);
  if (rc) return rc;
  const int64_t N = n_rows;
  float* loss_slot = grad_out + p->nparams;
  float* bias_slot = p->has_bias ? grad_out + p->fs.nfelem : nullptr;
  const float* bias = p->has_bias ? params + p->fs.nfelem : nullptr;
  const int reverse = (int)(p->parity & 1u);
  p->parity++;

  if (p->fused) {
    if (yhat_out != nullptr)  // the single-pass kernel does not emit y_hat; one extra forward pass
      TR_HIP(launch_rows(1, MODE_LIN_PRED, p->W, X, N, p->P, p->xld, p->dense, bias, nullptr, nullptr, 0.f, yhat_out,
                         nullptr, nullptr, stop_flag, st));
    const int64_t rpw = (N + p->fgrid - 1) / p->fgrid;
    {
      TimedLaunch tl(p, st, TR_KERNEL_STREAM_FUSED);
      TR_HIP(launch_linear_fused(p->fT, p->fCH, p->fgrid, X, N, p->P, p->xld, p->dense, bias, (const float*)target,
                                 (float)(2.0 / norm), p->gpart, p->dpart, yhat_out, rpw, reverse, stop_flag, st));
    }
    {
      TimedLaunch tl(p, st, TR_KERNEL_REDUCE);
      TR_HIP(launch_reduce_slabs(4, p->gpart, p->fgrid, p->P, p->G, p->dpart, p->fgrid, 1.0 / norm, loss_slot,
                                 bias_slot, stop_flag, st));
    }
  } else if (p->cluster) {
    if (yhat_out != nullptr)
      TR_HIP(launch_rows(1, MODE_LIN_PRED, p->W, X, N, p->P, p->xld, p->dense, bias, nullptr, nullptr, 0.f, yhat_out,
                         nullptr, nullptr, stop_flag, st));
    const int64_t rpc = (N + p->cncl - 1) / p->cncl;
    if ((uint64_t)p->cl_tag + (uint64_t)rpc + 2 >= 0xFFFFFFFFull) {  // tags would wrap: start over
      TR_HIP(hipMemsetAsync(p->gran, 0, (size_t)p->gran_n * 8, st));
      p->cl_tag = 0;
    }
    const uint32_t tag0 = p->cl_tag + 1;
    p->cl_tag += (uint32_t)rpc + 1;
    {
      TimedLaunch tl(p, st, TR_KERNEL_STREAM_FUSED);
      TR_HIP(launch_linear_cluster(p->cCH, p->cS, p->cncl, X, N, p->P, p->xld, p->dense, bias, (const float*)target,
                                   (float)(2.0 / norm), p->gpart, p->dpart, rpc, reverse, tag0, p->gran, p->err_word,
                                   stop_flag, st));
    }
    {
      TimedLaunch tl(p, st, TR_KERNEL_REDUCE);
      TR_HIP(launch_reduce_slabs(4, p->gpart, p->cncl, p->P, p->G, p->dpart, p->cncl, 1.0 / norm, loss_slot,
                                 bias_slot, stop_flag, st));
    }
  } else {
    const int C = p->C;
    TimedLaunch* tl_rows = new TimedLaunch(p, st, TR_KERNEL_STREAM_ROWS);
    if (p->model == TR_MODEL_LINEAR) {
      TR_HIP(launch_rows(1, MODE_LIN_TRAIN, p->W, X, N, p->P, p->xld, p->dense, bias, target, nullptr,
                         (float)(2.0 / norm), p->rowbuf, p->dpart, yhat_out, stop_flag, st));
    } else if (p->mfma_rows) {
      TR_HIP(launch_rows_mfma(MODE_MNL_TRAIN, X, N, p->P, p->xld, p->dense, C, (const int64_t*)target, class_weight,
                              (float)(1.0 / norm), p->rowbuf, p->dpart, stop_flag, st));
    } else {
      TR_HIP(launch_rows(C, MODE_MNL_TRAIN, p->W, X, N, p->P, p->xld, p->dense, nullptr, target, class_weight,
                         (float)(1.0 / norm), p->rowbuf, p->dpart, nullptr, stop_flag, st));
    }
    delete tl_rows;
    const int64_t nd = p->mfma_rows ? rows_mfma_num_waves(N) : rows_num_waves(C, N);
    const int cw = cols_cw(C);
    const int64_t PW = p->P / p->W;
    const int64_t nstripes = (PW + 256 * cw - 1) / (256 * cw);
    int64_t nchunks = (2048 + nstripes - 1) / nstripes;
    if (nchunks > p->max_slabs) nchunks = p->max_slabs;
    const int64_t by_rows = (N + 15) / 16;
    if (nchunks > by_rows) nchunks = by_rows;
    if (nchunks < 1) nchunks = 1;
    const int64_t rpc = (N + nchunks - 1) / nchunks;
    nchunks = (N + rpc - 1) / rpc;
    {
      TimedLaunch tl(p, st, TR_KERNEL_STREAM_COLS);
      TR_HIP(launch_cols(C, p->W, nstripes, nchunks, X, N, p->P, p->xld, p->rowbuf, rpc, p->gpart, 1, stop_flag, st));
    }
    {
      TimedLaunch tl(p, st, TR_KERNEL_REDUCE);
      TR_HIP(launch_reduce_slabs(p->W, p->gpart, nchunks, p->ncols, p->G, p->dpart, nd, 1.0 / norm, loss_slot,
                                 bias_slot, stop_flag, st));
    }
  }
  {
    TimedLaunch tl(p, st, TR_KERNEL_MTTKRP);
    TR_HIP(launch_mttkrp(p->fs, p->phi, p->dphi, weights, p->G, grad_out, stop_flag, st));
  }
  return 0;
}

static UpdateArgs make_args(float lambda_l2) {
  UpdateArgs ua;
  std::memset(&ua, 0, sizeof(ua));
  ua.lambda_l2 = lambda_l2;
  ua.bc2_sqrt = 1.f;
  return ua;
}

extern "C" int tr_finalize_grad(tr_plan* p, const float* params, const float* grad, float lambda_l2,
                                float* grad_total_out, float* loss_out, void* stream) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (params == nullptr || grad == nullptr || grad_total_out == nullptr) return fail(TR_E_ARG, "NULL buffer");
  TR_HIP(hipSetDevice(p->device));
  UpdateArgs ua = make_args(lambda_l2);
  ua.mode = 1;
  TR_HIP(launch_update(p->fs, p->has_bias, const_cast<float*>(params), grad, ua, nullptr, nullptr, nullptr,
                       grad_total_out, loss_out, nullptr, nullptr, (hipStream_t)stream));
  return 0;
}

extern "C" int tr_adam_step(tr_plan* p, float* params, const float* grad, float* exp_avg, float* exp_avg_sq,
                            float* max_exp_avg_sq, float lambda_l2, double lr, double beta1, double beta2,
                            double eps, double weight_decay, int amsgrad, int64_t step, double* loss_hist,
                            int64_t hist_base, int64_t iter, int64_t patience, double tol, int32_t* stop_flag,
                            void* stream) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  if (params == nullptr || grad == nullptr || exp_avg == nullptr || exp_avg_sq == nullptr)
    return fail(TR_E_ARG, "NULL buffer");
  if (amsgrad && max_exp_avg_sq == nullptr) return fail(TR_E_ARG, "amsgrad needs max_exp_avg_sq");
  if (step < 1) return fail(TR_E_ARG, "step must be >= 1");
  TR_HIP(hipSetDevice(p->device));
  UpdateArgs ua = make_args(lambda_l2);
  ua.mode = 0;
  ua.amsgrad = amsgrad ? 1 : 0;
  // torch/optim/adam.py (non-capturable): python-float arithmetic, then fp32 scalars
  const double st = (double)step;
  const double bc1 = 1.0 - std::pow(beta1, st);
  const double bc2 = 1.0 - std::pow(beta2, st);
  ua.step_size = (float)(lr / bc1);
  ua.bc2_sqrt = (float)std::pow(bc2, 0.5);
  ua.one_minus_b1 = (float)(1.0 - beta1);
  ua.beta2 = (float)beta2;
  ua.one_minus_b2 = (float)(1.0 - beta2);
  ua.eps = (float)eps;
  ua.weight_decay = (float)weight_decay;
  ua.hist_base = hist_base;
  ua.iter = iter;
  ua.patience = patience;
  ua.tol = tol;
  ua.nan_stop = p->model == TR_MODEL_SPECTRAL;  // spectral fit_Adam's NaN stop (spectral…py:738-741)
  // fold the next iteration's factor preparation into this launch (tr_plan_set_prepare_next)
  PrepArgs pa;
  std::memset(&pa, 0, sizeof(pa));
  if (p->prep_next && p->mnl && update_prepare_mode_ok(p->fs, 1)) {
    pa.mode = 1;
    pa.beta = p->sp_beta;
    pa.thr = p->sp_thr;
    pa.phi = p->phi;
    pa.dphi = p->dphi;
  }
  p->prepared = 0;
  TimedLaunch tl(p, (hipStream_t)stream, TR_KERNEL_UPDATE);
  TR_HIP(launch_update(p->fs, p->has_bias, params, grad, ua, exp_avg, exp_avg_sq, max_exp_avg_sq, nullptr, nullptr,
                       loss_hist, stop_flag, (hipStream_t)stream, &pa));
  if (pa.mode > 0) {
    p->prepared = 1;
    p->prep_params = params;
  }
  return 0;
}

extern "C" int tr_plan_status(tr_plan* p, int32_t* status) {
  if (p == nullptr || status == nullptr) return fail(TR_E_ARG, "NULL argument");
  *status = 0;
  if (p->err_word == nullptr) return 0;
  TR_HIP(hipSetDevice(p->device));
  uint32_t w = 0;
  TR_HIP(hipMemcpy(&w, p->err_word, 4, hipMemcpyDeviceToHost));  // synchronises the device
  if (w != 0) TR_HIP(hipMemset(p->err_word, 0, 4));
  *status = (int32_t)w;
  return 0;
}

extern "C" int tr_plan_set_timing(tr_plan* p, int enable) {
  if (p == nullptr) return fail(TR_E_ARG, "plan is NULL");
  p->timing = enable;  // bit mask over TR_KERNEL_* kinds (any non-zero value enables those bits)
  return 0;
}

extern "C" int tr_plan_read_timing(tr_plan* p, double* total_ms, int64_t* launches) {
  if (p == nullptr || total_ms == nullptr || launches == nullptr) return fail(TR_E_ARG, "NULL argument");
  for (int k = 0; k < TR_KERNEL_NKINDS; ++k) {
    total_ms[k] = 0.0;
    launches[k] = 0;
  }
  TR_HIP(hipSetDevice(p->device));
  for (auto& r : p->recs) {
    TR_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    TR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    if (r.kind >= 0 && r.kind < TR_KERNEL_NKINDS) {
      total_ms[r.kind] += ms;
      launches[r.kind] += 1;
    }
    p->pool.push_back(r.a);
    p->pool.push_back(r.b);
  }
  p->recs.clear();
  return 0;
}
