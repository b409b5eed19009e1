// ggnn_api.hip -- host side of libggnn.so: buffer layouts, kernel dispatch and
// the C ABI declared in include/ggnn.h.  Kernels: k_prep.h, k_prop.h, k_gru.h,
// k_wgrad.h.  See DESIGN.md for the HBM layout and the roofline per kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/ggnn.h"
#include "ggnn_common.h"
#include "k_gru.h"
#include "k_gru2.h"
#include "k_fused.h"
#include "k_prep.h"
#include "k_prop.h"
#include "k_optim.h"
#include "k_wgrad.h"
#include "k_head.h"
#include "k_gemm.h"
#include "k_gemm_ring.h"
#include "k_generic.h"
#include "k_pairs.h"

// ---------------------------------------------------------------------------
// error handling (thread-local last error; no exception crosses the ABI)
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                      \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) return fail(GGNN_ELAUNCH, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define LAUNCHCHK()                                                                                    \
  do {                                                                                                 \
    hipError_t e_ = hipGetLastError();                                                                 \
    if (e_ != hipSuccess) return fail(GGNN_ELAUNCH, std::string("launch: ") + hipGetErrorString(e_)); \
  } while (0)

namespace {

// ---- optional per-kernel-kind timing with HIP events (bench.py roofline)
const char* const kKindNames[GGNN_NUM_KERNEL_KINDS] = {
    "pack_weights", "prep_adjacency", "state_io", "prop_fwd", "gru_fwd", "gru_bwd", "prop_bwd", "wgrad", "optimizer",
    "heads", "fwd_fused"};
enum { K_PACK = 0, K_ADJ, K_IO, K_PROP_FWD, K_GRU_FWD, K_GRU_BWD, K_PROP_BWD, K_WGRAD, K_OPT, K_HEADS, K_FWD_FUSED };
struct ProfState {
  bool on = false;
  int cap = 0, used = 0;
  std::vector<hipEvent_t> ev;  // 2 per record
  std::vector<int> kind;
};
ProfState g_prof;
struct Prof {
  int idx = -1;
  hipStream_t s;
  Prof(int k, hipStream_t st) : s(st) {
    if (k >= 0 && g_prof.on && g_prof.used < g_prof.cap) {
      // (no records inside a hipGraph capture: the events would time the capture)
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
      idx = g_prof.used++;
      g_prof.kind[idx] = k;
      (void)hipEventRecord(g_prof.ev[2 * idx], s);
    }
  }
  ~Prof() {
    if (idx >= 0) (void)hipEventRecord(g_prof.ev[2 * idx + 1], s);
  }
};

// ---- configuration
struct Cfg {
  int b, vin, V, H, C, T, flags;
  int prec;  // PREC_BF16 / PREC_F16 / PREC_SPLIT
  bool split;
  long N;
  int act;  // bytes per stored activation element
  int vsh;  // log2(V)
  Drop edrop, sdrop;  // edge-weight / state dropout (thr == 0: off)
  bool ed, sd;
  bool generic;       // the general path (generic_path.h)
  bool sparse;        // GGNN_SPARSE_PAIRS (k_pairs.h)
  long pcap;          // pair-row capacity (sparse): 4 * b * v + PAIR_TILE * C, a multiple of PAIR_TILE
};

// seed_ptr (GGNN_SEED_DEVICE): `seed` is the address of a device uint64 read
// by the kernels at run time
Drop make_drop(float keep, uint64_t seed, bool seed_ptr = false) {
  Drop d;
  d.kp = seed_ptr ? (const uint32_t*)(uintptr_t)seed : nullptr;
  d.k0 = seed_ptr ? 0u : (uint32_t)seed;
  d.k1 = seed_ptr ? 0u : (uint32_t)(seed >> 32);
  if (keep >= 1.0f) {
    d.thr = 0;
    d.scale = 1.0f;
  } else {
    const double t = std::floor((double)keep * 4294967296.0);
    d.thr = (uint32_t)std::max(1.0, std::min(t, 4294967295.0));
    d.scale = 1.0f / keep;
  }
  return d;
}

int pad_v(int v) { return v <= 32 ? 32 : v <= 64 ? 64 : v <= 128 ? 128 : -1; }

int make_cfg(const ggnn_dims* d, Cfg* c) {
  if (!d) return fail(GGNN_EINVAL, "dims is NULL");
  if (d->b < 1 || d->v < 1 || d->C < 1 || d->T < 1) return fail(GGNN_EINVAL, "dims: b, v, C, T must be >= 1");
  if (d->h < 1 || d->h > 4096) return fail(GGNN_EUNSUP, "hidden size must lie in 1..4096 (got " + std::to_string(d->h) + ")");
  if (d->flags & ~(GGNN_USE_EDGE_BIAS | GGNN_FP32_PARITY | GGNN_FP16 | GGNN_DENSE_CHANNELS | GGNN_GENERIC |
                   GGNN_UNFUSED_FWD | GGNN_SPARSE_PAIRS | GGNN_SEED_DEVICE))
    return fail(GGNN_EINVAL, "unknown flag bits");
  // the specialised kernels: hidden 128 / 256, v <= 128; everything else runs
  // the general path (generic_path.h); pair mode is part of it
  c->sparse = (d->flags & GGNN_SPARSE_PAIRS) != 0;
  if (c->sparse && d->h % 4) return fail(GGNN_EUNSUP, "GGNN_SPARSE_PAIRS needs hidden % 4 == 0");
  c->generic = c->sparse || (d->flags & GGNN_GENERIC) || !(d->h == 128 || d->h == 256) || d->v > 128;
  c->pcap = c->sparse ? 4L * d->b * d->v + (long)PAIR_TILE * d->C : 0;
  const int V = c->generic ? d->v : pad_v(d->v);
  if (d->C > CHL_MAXC) return fail(GGNN_EUNSUP, "C must be <= " + std::to_string(CHL_MAXC));
  if ((d->flags & GGNN_FP32_PARITY) && (d->flags & GGNN_FP16))
    return fail(GGNN_EINVAL, "GGNN_FP32_PARITY and GGNN_FP16 are exclusive");
  c->b = d->b; c->vin = d->v; c->V = V; c->H = d->h; c->C = d->C; c->T = d->T; c->flags = d->flags;
  c->prec = (d->flags & GGNN_FP32_PARITY) ? PREC_SPLIT : (d->flags & GGNN_FP16) ? PREC_F16 : PREC_BF16;
  c->split = c->prec == PREC_SPLIT;
  c->act = c->split ? 4 : 2;
  c->N = (long)d->b * V;
  c->vsh = V == 32 ? 5 : V == 64 ? 6 : V == 128 ? 7 : 0;
  if (!(d->edge_keep > 0.0f && d->edge_keep <= 1.0f) || !(d->state_keep > 0.0f && d->state_keep <= 1.0f))
    return fail(GGNN_EINVAL, "dropout keep probabilities must lie in (0, 1] (edge_keep " +
                                 std::to_string(d->edge_keep) + ", state_keep " + std::to_string(d->state_keep) + ")");
  const bool sp = (d->flags & GGNN_SEED_DEVICE) != 0;
  if (sp && !d->seed && (d->edge_keep < 1.0f || d->state_keep < 1.0f))
    return fail(GGNN_EINVAL, "GGNN_SEED_DEVICE with dropout needs a device seed address in dims.seed");
  c->edrop = make_drop(d->edge_keep, d->seed, sp);
  c->sdrop = make_drop(d->state_keep, d->seed, sp);
  c->ed = c->edrop.thr != 0;
  c->sd = c->sdrop.thr != 0;
  if (!c->generic && (double)c->N * c->H * 4 >= 2147483647.0)
    return fail(GGNN_EUNSUP, "b*v*h too large for 32-bit buffer offsets");
  return GGNN_OK;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// ---- weight pack: bf16 hi part then lo part of every packed operand
// Under edge-weight dropout Wf / WT hold one masked copy per timestep
// (szW bytes apart).
// A pack serves every batch shape of one hidden size (bucketed batches have
// different v), so it holds the specialised kernels' fragment layouts when the
// hidden size has them (fast) AND the general path's fp32 copies.
struct PackL {
  bool fast;
  size_t Wf, WT, beta, Wg, WgT, Wc, WcT, bg, bc, szW;
  size_t gW, gszW, gWg, gWc, chocc, total;  // general path: fp32 W (per timestep under edge dropout), Wg, Wc;
                                            // chocc: the batch's channel occupancy (ggnn_pack_weights_batch)
  size_t gbits, gszB;  // edge dropout: the masked copies' keep bits per timestep (the pair dW product's mbits)
  long loW, loWg, loWc;  // element offset of the lo part from the hi part
  size_t wf(int t) const { return Wf + (size_t)t * szW; }
  size_t wt(int t) const { return WT + (size_t)t * szW; }
  size_t gw(int t) const { return gW + (size_t)t * gszW; }
  size_t gb(int t) const { return gbits + (size_t)t * gszB; }
};
PackL pack_layout(const Cfg& c) {
  PackL L;
  memset(&L, 0, sizeof(L));
  size_t o = 0;
  const size_t H = c.H;
  L.fast = (c.H == 128 || c.H == 256) && !(c.flags & GGNN_GENERIC);
  L.loW = (long)c.C * H * H;
  L.loWg = (long)4 * H * H;
  L.loWc = (long)2 * H * H;
  const int nW = c.ed ? c.T : 1;
  if (L.fast) {
    L.szW = al(2 * c.C * H * H * 2);
    L.Wf = o;   o += L.szW * nW;
    L.WT = o;   o += L.szW * nW;
    L.Wg = o;   o += al(2 * 4 * H * H * 2);
    L.WgT = o;  o += al(2 * 4 * H * H * 2);
    L.Wc = o;   o += al(2 * 2 * H * H * 2);
    L.WcT = o;  o += al(2 * 2 * H * H * 2);
  }
  L.beta = o; o += al(c.C * H * 4);
  L.bg = o;   o += al(2 * H * 4);
  L.bc = o;   o += al(H * 4);
  L.gszW = al((size_t)c.C * H * H * 4);
  L.gW = o;   o += L.gszW * nW;
  L.gWg = o;  o += al(4 * H * H * 4);
  L.gWc = o;  o += al(2 * H * H * 4);
  L.chocc = o; o += al(c.C);
  if (c.ed) {
    L.gszB = (size_t)c.C * H * ((H + 31) / 32) * 4;
    L.gbits = o; o += al(L.gszB * c.T);
  }
  L.total = o;
  return L;
}

// ---- staged adjacency
struct AdjL {
  size_t Ab, AbT, deg, chl, chl_all, occ, cgl, total;
};
AdjL adj_layout(const Cfg& c) {
  AdjL L;
  size_t o = 0;
  L.Ab = o;  o += al((size_t)c.b * c.C * c.V * c.V * 2);
  L.AbT = o; o += al((size_t)c.b * c.C * c.V * c.V * 2);
  L.deg = o; o += al((size_t)c.b * c.C * c.V * 2);
  L.chl = o; o += al((size_t)c.b * (c.C + 1) * 4);  // per-graph non-empty channel lists (k_chan_list)
  L.chl_all = o; o += al((size_t)(c.C + 1) * 4);     // identity list (dense channel loop)
  L.occ = o; o += al((size_t)c.b * c.C);              // (graph, channel) occupancy bytes
  L.cgl = o; o += al((size_t)c.C * (c.b + 1) * 4);    // per-channel graph lists (k_chan_graphs)
  L.total = o;
  return L;
}

// ---- per-batch workspace
struct WsL {
  size_t hb[2], Xa, hf[2];        // state (fp32 master; bf16 operand copy in bf16 mode)
  size_t hfT, hT, XT, rhT, r, u, c;  // saved per step (training)
  size_t dA, dB, dXT, dzcT, dzgT, dMT, dbp, gmax, wpart, gbp, sump, sbits;
  size_t nh4, nha, nhw;            // bytes of one [N][H] fp32 / activation / wgrad-operand array
  size_t total;
};
// the weight-gradient launch's plan (k_wgrad / k_wgrad256): output tile size,
// K chunk and chunk count of the T-summed problems, tiles, and -- under edge
// dropout -- the dW problem's timestep-aligned chunks: cpt chunks of KCt rows
// per timestep, each inside ONE timestep, so k_wgrad_reduce can apply the
// timestep's mask to the sum of its chunks (round 6: replaces the per-timestep
// dW tiles, their fp32 G scratch and k_edge_mask_reduce)
struct WgPlan {
  int TS;
  long KC, nchunks, tiles;
  long cpt, KCt;  // edge dropout only (else 0)
  long wgs;       // workgroups of the launch = partial tiles in the workspace
};
long wg256_kc(const Cfg& c);
WgPlan wg_plan(const Cfg& c) {
  WgPlan w;
  const long N = c.N, H = c.H;
  const bool big = H == 256 && N % 128 == 0;
  w.TS = big ? 256 : 128;
  const long t2 = (H / w.TS) * (H / w.TS);
  w.tiles = (6 + c.C) * t2;
  if (big) {
    w.KC = wg256_kc(c);
  } else {
    long KC = 4096;
    while (KC > 32 && (N % KC) != 0) KC /= 2;
    while (KC > 256 && w.tiles * (N / KC) < 256) KC /= 2;
    w.KC = KC;
  }
  w.nchunks = std::max<long>(N / std::max<long>(w.KC, 1), 1);
  w.cpt = w.KCt = 0;
  long dw_chunks = w.nchunks;
  if (c.ed) {
    // about as many chunks as the T-summed problems have (the same work per
    // workgroup): the smallest power of two >= nchunks / T whose chunk is a
    // whole number of 32-row slices, else one chunk per timestep.  (At
    // config 3 the 20 chunks per channel tile put the C channels' workgroups
    // of one chunk -- which read the same h_t^T rows -- on different XCDs:
    // +170 MB of HBM reads, L2 hit rate 0.50 -> 0.44, PMC
    // profiles/r06j_pmc_dropout_*.txt; 40 chunks, a multiple of the 8 XCDs,
    // took two rounds of workgroups and measured slower: wgrad 0.333 -> 0.350
    // ms per step, profiles/r06k_ab_cfg3_dw_chunks.log)
    long cpt = 1;
    while (cpt * c.T < w.nchunks && N % (cpt * 2 * 32) == 0) cpt *= 2;
    w.cpt = cpt;
    w.KCt = N / cpt;
    dw_chunks = (long)c.T * cpt;
  }
  w.wgs = 6 * t2 * w.nchunks + (long)c.C * t2 * dw_chunks;
  return w;
}
// rows of k_gru_bwd's per-workgroup bias partials (one row per (timestep, workgroup))
long gru_bias_rows(const Cfg& c);
constexpr int SUM_RCS = 32;  // k_sum_rows' row chunks (at most)
// Builder of one k_sum_rows / k_sum_rows_fin pair (fixed-order column sums):
// jobs take consecutive pieces of the scratch at `scr` (SUM_RCS * E floats
// each at most)
static_assert(GGNN_MAX_HEADS <= SUMJ_MAX, "heads_backward adds one SumPlan job per head");
struct SumPlan {
  SumJobs sj;
  int nb = 0, nf = 0;
  float* scr;
  bool full = false;  // a job past SUMJ_MAX was refused (launch() then fails)
  SumJob spill;       // what a refused add() hands back (never launched)
  explicit SumPlan(float* scratch) : scr(scratch) { memset(&sj, 0, sizeof(sj)); }
  // rows (t, w): part + t * sT + w * sW + (e / Nc) * sC + e % Nc
  SumJob& add(const float* part, int T, int nw, long sT, long sW, long E, long Nc, long sC, float* o0, float* o1,
              long split, int accumulate = 0) {
    if (sj.count == SUMJ_MAX) {
      full = true;
      return spill;
    }
    SumJob& q = sj.j[sj.count];
    const long rows = (long)T * nw;
    q.part = part; q.T = T; q.nw = nw; q.sT = sT; q.sW = sW; q.E = E; q.Nc = Nc; q.sC = sC;
    q.split = split; q.out0 = o0; q.out1 = o1; q.add = accumulate;
    q.rcs = (int)std::max<long>(1, std::min<long>(SUM_RCS, rows / 16));
    q.scratch = scr;
    scr += (long)q.rcs * E;
    sj.bx[sj.count] = nb;
    sj.fx[sj.count++] = nf;
    nb += (int)((E + 63) / 64) * q.rcs;
    nf += (int)((E + 255) / 256);
    return q;
  }
  // rows of E contiguous columns, row (t, w) at part + (t * stride + w) * E
  SumJob& rows(const float* part, int T, int nw, long stride, long E, float* o0, float* o1, long split) {
    return add(part, T, nw, stride * E, E, E, E, 0, o0, o1, split);
  }
  // GGNN_OK, or an error (nothing launched) when more than SUMJ_MAX jobs were added
  int launch(hipStream_t s) {
    if (full) return fail(GGNN_EINVAL, "k_sum_rows: more than " + std::to_string(SUMJ_MAX) + " sum jobs");
    if (!sj.count) return GGNN_OK;
    sj.bx[sj.count] = nb;
    sj.fx[sj.count] = nf;
    hipLaunchKernelGGL(k_sum_rows, dim3(nb), dim3(256), 0, s, sj);
    hipLaunchKernelGGL(k_sum_rows_fin, dim3(nf), dim3(256), 0, s, sj);
    return GGNN_OK;
  }
};
// k_slab_reduce over groups of z (GemmArgs::slab)
// workspace bytes of the gradient-scale word and k_absmax's block maxima
constexpr size_t GMAX_BYTES = 256 + ABSMAX_BLOCKS * 4;
// *gmax = max |x| over n floats as bits (k_absmax + k_absmax_fin; the block
// maxima 256 bytes past gmax)
void absmax(const float* x, long n, uint32_t* gmax, hipStream_t s) {
  float* part = (float*)((char*)gmax + 256);
  hipLaunchKernelGGL(k_absmax, dim3(ABSMAX_BLOCKS), dim3(ABSMAX_THREADS), 0, s, x, n, part);
  hipLaunchKernelGGL(k_absmax_fin, dim3(1), dim3(64), 0, s, (const float*)part, ABSMAX_BLOCKS, gmax);
}
void slab_launch(const SlabRed& r, hipStream_t s) {
  const long n = (long)r.M * r.N;
  const bool v4 = r.N % 4 == 0 && r.sSlab % 4 == 0 && (r.zT * r.sSlab) % 4 == 0 && ((uintptr_t)r.slab & 15) == 0;
  if (v4) hipLaunchKernelGGL(k_slab_reduce<4>, dim3((unsigned)((n / 4 + 255) / 256), (unsigned)r.G), dim3(256), 0, s, r);
  else hipLaunchKernelGGL(k_slab_reduce<1>, dim3((unsigned)((n + 255) / 256), (unsigned)r.G), dim3(256), 0, s, r);
}
void slab_reduce(const GemmArgs& a, int G, int zper, const int* zs, int sole, int add, long sDg, hipStream_t s) {
  SlabRed r;
  memset(&r, 0, sizeof(r));
  r.slab = a.slab; r.sSlab = a.sSlab; r.D = a.D; r.sDg = sDg; r.sDm = a.sDm;
  r.M = a.M; r.N = a.N; r.G = G; r.zper = zper; r.zs = zs; r.zsdiv = 1; r.nt = 1; r.zmask = a.zmask;
  r.sole = sole; r.add = add;
  slab_launch(r, s);
}
// the same over nt per-timestep slab sets of zT z's each, group g's z in
// [zs[g] / zsdiv, zs[g+1] / zsdiv) (stored, not added)
void slab_reduce_t(const GemmArgs& a, int G, const int* zs, int zsdiv, int nt, long zT, hipStream_t s,
                   const uint32_t* ugmax = nullptr) {
  SlabRed r;
  memset(&r, 0, sizeof(r));
  r.slab = a.slab; r.sSlab = a.sSlab; r.zT = zT; r.D = a.D; r.sDg = (long)a.M * a.N; r.sDm = a.sDm;
  r.M = a.M; r.N = a.N; r.G = G; r.zs = zs; r.zsdiv = zsdiv; r.nt = nt; r.ugmax = ugmax;
  const long n = (long)r.M * r.N;
  const bool v4 = r.N % 4 == 0 && r.sSlab % 4 == 0 && (r.zT * r.sSlab) % 4 == 0 && ((uintptr_t)r.slab & 15) == 0;
  if (v4) hipLaunchKernelGGL(k_seg_reduce<4>, dim3((unsigned)((n / 4 + 3) / 4), (unsigned)G), dim3(256), 0, s, r);
  else hipLaunchKernelGGL(k_seg_reduce<1>, dim3((unsigned)((n + 3) / 4), (unsigned)G), dim3(256), 0, s, r);
}

// the whole T-step forward of each graph in one workgroup (k_fused.h)
bool fused_fwd(const Cfg& c) {
  return !c.generic && c.H == 256 && c.V == 128 && c.T <= FUSED_MAXT && !(c.flags & GGNN_UNFUSED_FWD);
}
// training under state dropout on the fused forward: it writes the keep bits of
// every timestep's state mask (FusedFwdArgs::sbits), which the backward reads
bool state_bits(const Cfg& c) { return c.sd && fused_fwd(c); }
WsL ws_layout(const Cfg& c, bool training) {
  WsL L;
  memset(&L, 0, sizeof(L));
  size_t o = 0;
  const size_t N = c.N, H = c.H, T = c.T, C = c.C;
  L.nh4 = al(N * H * 4);
  L.nha = al(N * H * c.act);
  const size_t nh2 = al(N * H * 2);
  L.nhw = nh2;
  if (!c.split) {
    L.hb[0] = o; o += nh2;
    L.hb[1] = o; o += nh2;
  }
  L.Xa = o; o += L.nh4;  // fp32 X scratch of the fused forward (k_fused.h) in every mode; 16-bit X otherwise
  if (!training) {
    L.hf[0] = o; o += L.nh4;
    L.hf[1] = o; o += L.nh4;
  } else {
    L.hfT = o; o += L.nh4 * (T + 1);
    L.hT = o;  o += L.nhw * T;
    L.XT = o;  o += L.nhw * T;
    L.rhT = o; o += L.nhw * T;
    L.r = o;   o += L.nh4 * T;
    L.u = o;   o += L.nh4 * T;
    L.c = o;   o += L.nh4 * T;
    L.dA = o;  o += L.nh4;
    L.dB = o;  o += L.nh4;
    L.dXT = o; o += L.nha;
    L.dzcT = o; o += L.nhw * T;
    L.dzgT = o; o += 2 * L.nhw * T;
    L.dMT = o;  o += C * L.nhw * T;
    L.dbp = o; o += al(T * (size_t)c.b * C * H * 4);    // per-(timestep, graph) dL/dbeta partials
    L.gmax = o; o += al(GMAX_BYTES);                      // max |dL/dh_T| (gradient scale, ggnn_common.h) + k_absmax partials
    if (H >= 128) {                                       // deterministic K-chunk reduction of the weight gradients
      const WgPlan w = wg_plan(c);
      L.wpart = o; o += al((size_t)w.wgs * w.TS * w.TS * 4);
    }
    L.gbp = o; o += al((size_t)gru_bias_rows(c) * 3 * H * 4);  // k_gru_bwd's [dbg | dbc] partials
    L.sump = o; o += al((size_t)SUM_RCS * (3 * H + C * H) * 4);  // k_sum_rows' per-row-chunk sums
    // the state keep bits [T][b][512 threads] uint2 (state_bits): laid out
    // whenever the fused forward runs, whatever the keep probabilities, so a
    // workspace sized without state dropout still holds them (5 MiB at config 3)
    L.sbits = 0;
    if (fused_fwd(c)) { L.sbits = o; o += al((size_t)T * c.b * 512 * 8); }
  }
  L.total = o;
  return L;
}

template <typename T> T* P(void* base, size_t off) { return (T*)((char*)base + off); }
template <typename T> const T* P(const void* base, size_t off) { return (const T*)((const char*)base + off); }
// the channel list the compute kernels loop over: per-graph non-empty
// channels (graph stride C+1), or the identity list (stride 0) under
// GGNN_DENSE_CHANNELS
struct ChanL {
  const int* p;
  int stride;
};
ChanL chan_lists(const Cfg& c, const void* adj, const AdjL& AL) {
  if (c.flags & GGNN_DENSE_CHANNELS) return ChanL{P<int>(adj, AL.chl_all), 0};
  return ChanL{P<int>(adj, AL.chl), c.C + 1};
}
int grid1d(long n, int bs = 256) {
  const long g = (n + bs - 1) / bs;
  return (int)std::min<long>(std::max<long>(g, 1), 8192);
}
// device-side fill / copy on the stream (kernels: one kind of graph node
// under stream capture; tools/build_memset_probe_lib.py builds the round-2
// hipMemsetAsync / hipMemcpyAsync form for tools/capture_probe.py)
void fill_async(void* p, unsigned char byte, size_t nbytes, hipStream_t s) {
  if (!nbytes) return;
  hipLaunchKernelGGL(k_fill, dim3(grid1d((long)((nbytes + 15) / 16))), dim3(256), 0, s, (unsigned char*)p, nbytes,
                     (unsigned)byte);
}
// up to FILL_MAXJ fills as one launch (empty fills skipped)
struct FillSet {
  FillJobs f;
  int count = 0;
  size_t maxn = 0;
  void add(void* p, unsigned char byte, size_t nbytes) {
    if (!nbytes) return;
    f.p[count] = (unsigned char*)p; f.n[count] = nbytes; f.byte[count] = byte;
    ++count;
    maxn = std::max(maxn, nbytes);
  }
  void launch(hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(k_fill_multi, dim3(grid1d((long)((maxn + 15) / 16)), count), dim3(256), 0, s, f);
  }
};
void copy_async(float* dst, const float* src, long n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy32, dim3(grid1d((n + 3) / 4)), dim3(256), 0, s, dst, src, n);
}

// ---- dispatch helpers
// rows per GRU workgroup = 32*RT; RT capped per kernel by its VGPR budget
int gru_rt(const Cfg& c, int maxrt) {
  const long t = c.N / 32;
  if (maxrt >= 4 && t % 4 == 0) return 4;
  if (maxrt >= 2 && t % 2 == 0) return 2;
  return 1;
}

template <int V, int H, int PREC>
void launch_prop_fwd(const Cfg& c, int t, const void* hs, const u16* Ab, ChanL chl, const PackL& PL,
                     const void* pk, void* Xa, void* XT, hipStream_t s) {
  Prof p(K_PROP_FWD, s);
  hipLaunchKernelGGL((k_prop_fwd<V, H, PREC>), dim3(c.b), dim3(2 * H), 0, s, (const ActT<PREC>*)hs, Ab, chl.p, chl.stride,
                     P<u16>(pk, PL.wf(c.ed ? t : 0)), PL.loW, P<float>(pk, PL.beta), (ActT<PREC>*)Xa, (u16*)XT, c.C, c.N);
}
// k_wgrad256's K chunk at hidden 256 (one workgroup per CU, 128 KiB LDS
// ring): the largest chunk that still gives >= 7/8 of the CUs a tile-chunk;
// the problems hold 6 + C tiles of 256 x 256 (dWg 4, dWc 2, dW one per channel)
long wg256_kc(const Cfg& c) {
  const long N = c.N, tiles_eq = 6 + c.C;
  long KC = 8192;
  while (KC > 128 && ((N % KC) != 0 || tiles_eq * (N / KC) < 224)) KC /= 2;
  return KC;
}
// whether dW_c runs over channel c's graph list (k_chan_graphs) instead of
// every row: the specialised path at hidden 256 with channel skipping, when a
// K chunk's share of the graphs fits the kernel's register list.  Then
// k_prop_bwd writes no dM^T rows for a graph's empty channels.
bool wgrad_lists(const Cfg& c) {
  if (!(c.H == 256 && c.N % 128 == 0) || (c.flags & GGNN_DENSE_CHANNELS)) return false;
  const WgPlan w = wg_plan(c);
  const long per_t = c.ed ? w.cpt : w.nchunks;  // chunks a channel's graph list is split into
  return (c.b + per_t - 1) / per_t <= WG_LIST_MAX && c.V % 32 == 0;
}

// k_prop_bwd's dh += dM W_c^T with its limb corrections on the fp8 MFMA
// (ggnn_common.h mfma_f8corr): the fp32-parity mode, hidden a multiple of 32
bool prop_f8(const Cfg& c) { return c.prec == PREC_SPLIT && c.H % 32 == 0; }

template <int V, int H, int PREC>
void launch_prop_bwd(const Cfg& c, int t, const void* dXT, const u16* AbT, const u16* deg, ChanL chl,
                     const PackL& PL, const void* pk, const float* dh_in, float* dh_out, void* dMT, float* dbp,
                     const uint32_t* gmax, const uint2* sbits, hipStream_t s) {
  Prof p(K_PROP_BWD, s);
  // (the forward's state keep bits: 128-row graphs at hidden 256 only)
  hipLaunchKernelGGL((k_prop_bwd<V, H, PREC>), dim3(c.b), dim3(2 * H), 0, s, (const ActT<PREC>*)dXT, AbT, deg, chl.p,
                     chl.stride,
                     P<u16>(pk, PL.wt(c.ed ? t : 0)), PL.loW, dh_in, dh_out, (u16*)dMT, dbp, c.C, c.N, c.sdrop, t - 1,
                     gmax, (int)!wgrad_lists(c), (V == 128 && H == 256) ? sbits : (const uint2*)nullptr);
}
template <int H, int RT, int PREC>
void launch_gru_fwd(const Cfg& c, int t, const void* Xa, const u16* hb, const float* hf, const PackL& PL,
                    const void* pk, float* hf_out, u16* hb_out, void* hT, float* r, float* u, float* cc, void* rhT,
                    hipStream_t s) {
  Prof p(K_GRU_FWD, s);
  if constexpr (Prec<PREC>::split && H == 256) {
    // 128-row tiles with K-streamed activations (k_gru2.h)
    if (c.N % 128 == 0) {
      hipLaunchKernelGGL(k_gru_fwd2, dim3(c.N / 128), dim3(512), 0, s, (const float*)Xa, hf, P<u16>(pk, PL.Wg),
                         P<float>(pk, PL.bg), P<u16>(pk, PL.Wc), P<float>(pk, PL.bc), PL.loWg, PL.loWc, hf_out,
                         (u16*)hT, r, u, cc, (u16*)rhT, c.N, c.sdrop, t, c.vsh);
      return;
    }
  }
  hipLaunchKernelGGL((k_gru_fwd<H, RT, PREC>), dim3(c.N / (32 * RT)), dim3(2 * H), 0, s, (const ActT<PREC>*)Xa, hb,
                     hf, P<u16>(pk, PL.Wg), P<float>(pk, PL.bg), P<u16>(pk, PL.Wc), P<float>(pk, PL.bc), PL.loWg,
                     PL.loWc, hf_out, hb_out, (u16*)hT, r, u, cc, (u16*)rhT, c.N, c.sdrop, t, c.vsh);
}
template <int H, int RT, int PREC>
void launch_gru_bwd(const Cfg& c, const float* delta, const float* hf, const float* r, const float* u, const float* cc,
                    const PackL& PL, const void* pk, void* dXT, float* dh_out, void* dzcT, void* dzgT, float* dbc,
                    float* dbg, const uint32_t* gmax, float* bpart, const uint2* sbits, int* nwg, hipStream_t s) {
  Prof p(K_GRU_BWD, s);
  *nwg = (int)(c.N / (32 * RT));
  hipLaunchKernelGGL((k_gru_bwd<H, RT, PREC>), dim3(c.N / (32 * RT)), dim3(2 * H), 0, s, delta, hf, r, u, cc,
                     P<u16>(pk, PL.WcT), P<u16>(pk, PL.WgT), PL.loWc, PL.loWg, (ActT<PREC>*)dXT, dh_out,
                     (u16*)dzcT, (u16*)dzgT, dbc, dbg, c.N, gmax, bpart,
                     (H == 256 && c.V == 128) ? sbits : (const uint2*)nullptr, c.sdrop.scale);
}
long gru_bias_rows(const Cfg& c) { return (long)c.T * std::max<long>(c.N / 32, 1); }

#define DISPATCH_V(c, FN, H, PREC, ...)                 \
  do {                                                  \
    if ((c).V == 32) FN<32, H, PREC>(__VA_ARGS__);      \
    else if ((c).V == 64) FN<64, H, PREC>(__VA_ARGS__); \
    else FN<128, H, PREC>(__VA_ARGS__);                 \
  } while (0)
#define DISPATCH_VH(c, FN, PREC, ...)                                  \
  do {                                                                 \
    if ((c).H == 64) DISPATCH_V(c, FN, 64, PREC, __VA_ARGS__);         \
    else if ((c).H == 128) DISPATCH_V(c, FN, 128, PREC, __VA_ARGS__);  \
    else DISPATCH_V(c, FN, 256, PREC, __VA_ARGS__);                    \
  } while (0)
#define DISPATCH_RT(c, FN, H, PREC, ...)                                             \
  do {                                                                               \
    constexpr bool sp_ = Prec<PREC>::split;                                          \
    constexpr int mx_ = sp_ ? kSplitRT<FN##_tag>::value : kMaxRT<FN##_tag, H>::value; \
    const int rt_ = gru_rt(c, mx_);                                                  \
    if (mx_ >= 4 && rt_ == 4) FN<H, mx_ >= 4 ? 4 : 2, PREC>(__VA_ARGS__);            \
    else if (rt_ == 2) FN<H, 2, PREC>(__VA_ARGS__);                                  \
    else FN<H, 1, PREC>(__VA_ARGS__);                                                \
  } while (0)
#define DISPATCH_HRT(c, FN, PREC, ...)                                 \
  do {                                                                 \
    if ((c).H == 64) DISPATCH_RT(c, FN, 64, PREC, __VA_ARGS__);        \
    else if ((c).H == 128) DISPATCH_RT(c, FN, 128, PREC, __VA_ARGS__); \
    else DISPATCH_RT(c, FN, 256, PREC, __VA_ARGS__);                   \
  } while (0)

// RT caps: the fused GRU backward at H = 256 keeps a1/a2 (2 x 16 x RT fp32
// registers) live through both products and spills at RT = 4.
struct launch_gru_fwd_tag {};
struct launch_gru_bwd_tag {};
template <typename TAG, int H> struct kMaxRT { static constexpr int value = 4; };
template <typename TAG> struct kSplitRT { static constexpr int value = 2; };
template <> struct kMaxRT<launch_gru_bwd_tag, 256> { static constexpr int value = 2; };

void launch_pack(bool f16, const float* S, int ldS, long sS, int K, int N, int trans, u16* out, long sO, long lo,
                 int batch, hipStream_t s, Drop dr = Drop{0, 0, 0, 1.0f}, int t = 0) {
  const int total = (N / 32) * (K / 16) * 64;
  Prof p(K_PACK, s);
  if (f16)
    hipLaunchKernelGGL(k_pack_B<true>, dim3((total + 255) / 256, batch), dim3(256), 0, s, S, ldS, sS, K, N, trans, out,
                       sO, lo, dr, t);
  else
    hipLaunchKernelGGL(k_pack_B<false>, dim3((total + 255) / 256, batch), dim3(256), 0, s, S, ldS, sS, K, N, trans, out,
                       sO, lo, dr, t);
}
const Drop kNoDrop = {0, 0, 0, 1.0f};

// -------------------------------------------------------------------- forward
template <int PREC>
int forward_impl(const Cfg& c, const void* pack, const void* adj, void* ws, bool tr, const float* h0, float* hT,
                 hipStream_t s) {
  typedef ActT<PREC> Act;
  constexpr bool SPLIT = Prec<PREC>::split;
  const WsL L = ws_layout(c, tr);
  const PackL PL = pack_layout(c);
  const AdjL AL = adj_layout(c);
  const long N = c.N, H = c.H;
  // unpadded batch (v a multiple of 32): the caller's h0 / hT are the engine's
  // row layout, so inference reads h0 in place and the last step writes hT in
  // place (training copies h0: the backward needs it after the caller's buffer
  // may have changed)
  const bool dense = c.vin == c.V;
  // the whole T-step forward of each graph in one workgroup (k_fused.h)
  const bool fused = fused_fwd(c);
  float* hf0 = tr ? P<float>(ws, L.hfT) : P<float>(ws, L.hf[0]);
  if (tr) {
    Prof p(K_IO, s);
    hipLaunchKernelGGL((k_stage_h0<Prec<PREC>::f16>), dim3((N + 63) / 64, H / 64), dim3(256), 0, s, h0, c.vin, c.V,
                       hf0, SPLIT ? (u16*)nullptr : P<u16>(ws, L.hb[0]), P<u16>(ws, L.hT), N, c.H);
  } else if (!dense || (!SPLIT && !fused)) {
    Prof p(K_IO, s);
    hipLaunchKernelGGL(k_pad_state, dim3(grid1d(N / 4 * H)), dim3(256), 0, s, h0, c.vin, c.V, c.H,
                       dense ? (float*)nullptr : hf0, SPLIT ? (u16*)nullptr : P<u16>(ws, L.hb[0]), N,
                       (int)Prec<PREC>::f16, kNoDrop, 0, (const uint32_t*)nullptr);
  }
  if (fused) {
    FusedFwdArgs fa;
    memset(&fa, 0, sizeof(fa));
    fa.Ab = P<u16>(adj, AL.Ab);
    const ChanL cl = chan_lists(c, adj, AL);
    fa.chl = cl.p;
    fa.chs = cl.stride;
    fa.Wp = P<u16>(pack, PL.wf(0));
    fa.wlo = PL.loW;
    fa.wstep = c.ed ? (long)(PL.szW / 2) : 0;
    fa.beta = P<float>(pack, PL.beta);
    fa.Wgp = P<u16>(pack, PL.Wg);
    fa.bg = P<float>(pack, PL.bg);
    fa.Wcp = P<u16>(pack, PL.Wc);
    fa.bc = P<float>(pack, PL.bc);
    fa.wlo_g = PL.loWg;
    fa.wlo_c = PL.loWc;
    fa.Xs = P<float>(ws, L.Xa);
    for (int t = 0; t <= c.T; ++t) {
      const float* hin = tr ? P<float>(ws, L.hfT + L.nh4 * t) : (t == 0 && dense) ? h0 : P<float>(ws, L.hf[t & 1]);
      fa.hf[t] = (t == c.T && dense) ? hT : (float*)hin;
    }
    if (tr) {
      fa.XT = P<u16>(ws, L.XT);
      fa.hT = P<u16>(ws, L.hT);
      fa.rhT = P<u16>(ws, L.rhT);
      fa.r = P<float>(ws, L.r);
      fa.u = P<float>(ws, L.u);
      fa.c = P<float>(ws, L.c);
      fa.sw = (long)(L.nhw / 2);
      fa.s4 = (long)(L.nh4 / 4);
    }
    fa.C = c.C;
    fa.T = c.T;
    fa.vsh = c.vsh;
    fa.sd = c.sdrop;
    fa.sbits = (tr && state_bits(c)) ? P<uint2>(ws, L.sbits) : nullptr;
    {
      Prof p(K_FWD_FUSED, s);
      hipLaunchKernelGGL(k_fwd_fused<PREC>, dim3(c.b), dim3(512), 0, s, fa);
    }
  } else
  for (int t = 0; t < c.T; ++t) {
    const float* hf_in = tr ? P<float>(ws, L.hfT + L.nh4 * t)
                            : (t == 0 && dense) ? h0 : P<float>(ws, L.hf[t & 1]);
    float* hf_out = (t + 1 == c.T && dense) ? hT
                    : tr                   ? P<float>(ws, L.hfT + L.nh4 * (t + 1))
                                           : P<float>(ws, L.hf[(t + 1) & 1]);
    const u16* hb_in = SPLIT ? nullptr : P<u16>(ws, L.hb[t & 1]);
    u16* hb_out = SPLIT ? nullptr : P<u16>(ws, L.hb[(t + 1) & 1]);
    const void* hs = SPLIT ? (const void*)hf_in : (const void*)hb_in;
    void* XT = tr ? P<void>(ws, L.XT + L.nhw * t) : nullptr;
    DISPATCH_VH(c, launch_prop_fwd, PREC, c, t, hs, P<u16>(adj, AL.Ab), chan_lists(c, adj, AL), PL, pack,
                P<void>(ws, L.Xa), XT, s);
    void* hTo = (tr && t + 1 < c.T) ? P<void>(ws, L.hT + L.nhw * (t + 1)) : nullptr;
    float* ro = tr ? P<float>(ws, L.r + L.nh4 * t) : nullptr;
    float* uo = tr ? P<float>(ws, L.u + L.nh4 * t) : nullptr;
    float* co = tr ? P<float>(ws, L.c + L.nh4 * t) : nullptr;
    void* rhT = tr ? P<void>(ws, L.rhT + L.nhw * t) : nullptr;
    DISPATCH_HRT(c, launch_gru_fwd, PREC, c, t, P<void>(ws, L.Xa), hb_in, hf_in, PL, pack, hf_out, hb_out, hTo, ro, uo,
                 co, rhT, s);
  }
  const float* hfin = tr ? P<float>(ws, L.hfT + L.nh4 * c.T) : P<float>(ws, L.hf[c.T & 1]);
  if (!dense) {
    Prof p(K_IO, s);
    hipLaunchKernelGGL(k_unpad_state, dim3(grid1d((long)c.b * c.vin * H)), dim3(256), 0, s, hfin, c.vin, c.V, c.H, hT,
                       (long)c.b, (const uint32_t*)nullptr);
  }
  LAUNCHCHK();
  return GGNN_OK;
}

// ------------------------------------------------------------------- backward
template <int PREC>
int wgrad_impl(const Cfg& c, void* ws, int t0, int nt, float* dW, float* dWg, float* dWc, hipStream_t s);

// gradient accumulators zeroed by grouped k_zero_multi launches (flushed when
// the job table fills and on scope exit)
struct Zeroer {
  hipStream_t s;
  ZeroJobs j;
  int n = 0;
  explicit Zeroer(hipStream_t st) : s(st) {}
  void add(float* p, long cnt) {
    if (cnt <= 0) return;
    j.p[n] = p, j.n[n] = cnt;
    if (++n == ZERO_MAXJ) flush();
  }
  void flush() {
    if (n) hipLaunchKernelGGL(k_zero_multi, dim3(256, n), dim3(256), 0, s, j);
    n = 0;
  }
  ~Zeroer() { flush(); }
};

template <int PREC>
int backward_impl(const Cfg& c, const void* pack, const void* adj, void* ws, const float* dhT, float* dh0, float* dW,
                  float* dbeta, float* dWg, float* dbg, float* dWc, float* dbc, hipStream_t s) {
  const WsL L = ws_layout(c, true);
  const PackL PL = pack_layout(c);
  const AdjL AL = adj_layout(c);
  const long N = c.N, H = c.H;
  const bool use_bias = (c.flags & GGNN_USE_EDGE_BIAS) != 0;
  if (H < 128) return fail(GGNN_EUNSUP, "weight gradients need hidden >= 128");

  // (the weight and bias gradients need no clearing: k_wgrad_reduce and
  // k_sum_rows store every element once)
  // gradient scale: the backward runs on S * dL/dh_T, S = 2^-floor(log2 max|dL/dh_T|),
  // and divides its outputs by S (ggnn_common.h gscale): loss-normalised
  // gradients (~1/b) stay inside the f16 limbs' normal range
  const uint32_t* gmax = P<const uint32_t>(ws, L.gmax);
  {
    Prof p(K_IO, s);
    absmax(dhT, (long)c.b * c.vin * H, P<uint32_t>(ws, L.gmax), s);
  }
  float* dA = P<float>(ws, L.dA);
  float* dB = P<float>(ws, L.dB);
  // unpadded batch without state dropout: dL/dh_T is read in place and the
  // last step writes dL/dh0 in place
  const bool dense = c.vin == c.V;
  // the forward's state keep bits (state_bits): the first step applies the
  // last timestep's mask to dL/dh_T as it reads it, so it is read in place too
  const uint2* sb = state_bits(c) ? P<const uint2>(ws, L.sbits) : nullptr;
  const bool in_place = dense && (!c.sd || sb);
  if (!in_place) {
    Prof p(K_IO, s);
    hipLaunchKernelGGL(k_pad_state, dim3(grid1d(N / 4 * H)), dim3(256), 0, s, dhT, c.vin, c.V, c.H, dA, (u16*)nullptr, N, 0,
                       c.sdrop, c.T - 1, gmax);
  }
  const long gb_stride = std::max<long>(N / 32, 1);  // bias-partial rows per timestep (k_gru_bwd, RT = 1 bound)
  int gb_nwg = 0;
  for (int t = c.T - 1; t >= 0; --t) {
    const bool first = t == c.T - 1 && in_place, last = t == 0 && dense;
    const float* delta = first ? dhT : dA;
    float* dh_out = last ? dh0 : dA;
    DISPATCH_HRT(c, launch_gru_bwd, PREC, c, delta, P<float>(ws, L.hfT + L.nh4 * t), P<float>(ws, L.r + L.nh4 * t),
                 P<float>(ws, L.u + L.nh4 * t), P<float>(ws, L.c + L.nh4 * t), PL, pack, P<void>(ws, L.dXT), dB,
                 P<void>(ws, L.dzcT + L.nhw * t), P<void>(ws, L.dzgT + 2 * L.nhw * t), dbc, dbg,
                 first ? gmax : (const uint32_t*)nullptr, P<float>(ws, L.gbp) + (size_t)t * gb_stride * 3 * H,
                 (first && c.sd) ? sb + (size_t)t * c.b * 512 : (const uint2*)nullptr, &gb_nwg, s);
    DISPATCH_VH(c, launch_prop_bwd, PREC, c, t, P<void>(ws, L.dXT), P<u16>(adj, AL.AbT), P<u16>(adj, AL.deg),
                chan_lists(c, adj, AL), PL, pack,
                dB, dh_out, P<void>(ws, L.dMT + (size_t)c.C * L.nhw * t),
                use_bias ? P<float>(ws, L.dbp) + (size_t)t * c.b * c.C * c.H : nullptr,
                last ? gmax : (const uint32_t*)nullptr, sb, s);
  }
  // all weight gradients in one grouped launch over every timestep (measured:
  // 20 % faster than one launch per timestep right after its producers, whose
  // operands would still sit in the Infinity Cache)
  if (int e = wgrad_impl<PREC>(c, adj, ws, 0, c.T, dW, dWg, dWc, s)) return e;
  {
    Prof p(K_IO, s);
    if (!dense)
      hipLaunchKernelGGL(k_unpad_state, dim3(grid1d((long)c.b * c.vin * H)), dim3(256), 0, s, dA, c.vin, c.V, c.H, dh0,
                         (long)c.b, gmax);
    // bias gradients: fixed-order sums of the per-(timestep, graph) dbeta and
    // the per-(timestep, workgroup) GRU bias partials
    // (the sums and k_wgrad_reduce's stores carry the unscale 1 / S: no
    // separate pass over the gradients)
    SumPlan sp(P<float>(ws, L.sump));
    sp.rows(P<const float>(ws, L.gbp), c.T, gb_nwg, gb_stride, 3 * H, dbg, dbc, 2 * H).ugmax = gmax;
    if (use_bias)
      sp.rows(P<const float>(ws, L.dbp), 1, c.T * c.b, c.T * c.b, (long)c.C * H, dbeta, dbeta, (long)c.C * H).ugmax = gmax;
    if (int e = sp.launch(s)) return e;
  }

  LAUNCHCHK();
  return GGNN_OK;
}

// Weight gradients of timesteps [t0, t0 + nt): out[m][n] = sum_{t,rows}
// P_t[m][row] Q_t[n][row], one grouped launch (k_wgrad.h).  The outputs are
// STORED, not accumulated (k_wgrad_reduce writes each element once, already
// unscaled): the one caller passes all timesteps at once (t0 = 0, nt = T).
template <int PREC>
int wgrad_impl(const Cfg& c, const void* adj, void* ws, int t0, int nt, float* dW, float* dWg, float* dWc,
               hipStream_t s) {
  const WsL L = ws_layout(c, true);
  const long N = c.N, H = c.H;
  if (H < 128) return fail(GGNN_EUNSUP, "weight gradients need hidden >= 128");
  if (t0 != 0 || nt != c.T) return fail(GGNN_EINVAL, "weight gradients: stored over all timesteps at once");
  WgArgs a;
  memset(&a, 0, sizeof(a));
  int np = 0, tiles = 0;
  const long sa = (long)(L.nhw / 2);  // elements of one [H][N] weight-gradient operand array
  // 256x256 tiles (k_wgrad256) at hidden = 256: every problem has M = 256
  const bool big = H == 256 && N % 128 == 0;
  const int TS = big ? 256 : 128;
  const WgPlan wp = wg_plan(c);
  int wgs = 0;
  auto add = [&](size_t Poff, long stepP, size_t Qoff, long stepQ, float* out, int ldO, int M, int Nn, int nb = 1,
                 long sQb = 0, long sOb = 0) {
    WgProb& p = a.p[np++];
    p.P = P<u16>(ws, Poff) + (long)t0 * stepP;
    p.Q = P<u16>(ws, Qoff) + (long)t0 * stepQ;
    p.out = out;
    p.ldP = N; p.ldQ = N; p.stepP = stepP; p.stepQ = stepQ; p.sQb = sQb; p.sOb = sOb;
    p.ldO = ldO; p.M = M; p.N = Nn; p.tiles_n = Nn / TS; p.tiles_b = (M / TS) * p.tiles_n;
    p.sPb = 0; p.pdiv = 1; p.T = nt;
    p.tile_begin = tiles;
    tiles += nb * p.tiles_b;
    p.nch = (int)wp.nchunks;
    p.cpt = 0;
    p.KCt = 0;
    p.wg_begin = wgs;
    wgs += nb * p.tiles_b * p.nch;
  };
  // d gates_kernel: rows [0,H) from X, rows [H,2H) from h ; columns dzg (2H)
  add(L.XT, sa, L.dzgT, 2 * sa, dWg, 2 * H, H, 2 * H);
  add(L.hT, sa, L.dzgT, 2 * sa, dWg + H * 2 * H, 2 * H, H, 2 * H);
  // d candidate_kernel: rows [0,H) from X, rows [H,2H) from r*h ; columns dzc (H)
  add(L.XT, sa, L.dzcT, sa, dWc, H, H, H);
  add(L.rhT, sa, L.dzcT, sa, dWc + H * H, H, H, H);
  // d edge_weights[c] = sum_t mask_t/keep (h_t^T dM_{c,t}): one problem batched
  // over the C channels.  Under edge dropout its K chunks are timestep-aligned
  // (wp.cpt chunks of wp.KCt rows per timestep): k_wgrad_reduce sums each
  // timestep's chunks, applies that timestep's mask (Philox, as the pack drew
  // it) and adds the timesteps in order
  add(L.hT, sa, L.dMT, c.C * sa, dW, H, H, H, c.C, sa, (long)H * H);
  if (c.ed) {
    WgProb& q = a.p[np - 1];
    q.cpt = (int)wp.cpt;
    q.KCt = (int)wp.KCt;
    q.nch = (int)(nt * wp.cpt);
    wgs = q.wg_begin + c.C * q.tiles_b * q.nch;
    a.edrop = c.edrop;
  }
  constexpr int WP = WgradPrec<PREC>::value;
  a.nprob = np;
  a.H = (int)H;
  if (wp.tiles != tiles || wp.wgs != wgs || wp.TS != TS)
    return fail(GGNN_EINVAL, "weight gradients: launch plan and workspace disagree");
  // deterministic reduction over the K chunks (k_wgrad_reduce): the partial
  // tiles live in the workspace
  a.part = P<float>(ws, L.wpart);
  a.gmax = P<const uint32_t>(ws, L.gmax);  // outputs / S (the backward's gradient scale)
  if (big) {
    const long KC = wp.KC;
    if (N % KC || KC % 128) return fail(GGNN_EUNSUP, "rows not divisible into weight-gradient chunks");
    if (tiles != 6 + c.C) return fail(GGNN_EINVAL, "k_wgrad256: unexpected problem set");
    a.KC = (int)KC;
    a.nchunks = (int)(N / KC);
    if (wgrad_lists(c)) {
      // dW_c over the rows of channel c's graphs only (the last problem)
      WgProb& q = a.p[np - 1];
      q.gl = P<const int>(adj, adj_layout(c).cgl);
      q.gls = c.b + 1;
      q.glmod = c.C;
      q.V32 = c.V / 32;
    }
    Prof p(K_WGRAD, s);
    hipLaunchKernelGGL((k_wgrad256<WP>), dim3(wgs), dim3(512), 0, s, a);
    hipLaunchKernelGGL(k_wgrad_reduce<256>, dim3(tiles * 64), dim3(256), 0, s, a);
    return GGNN_OK;
  }
  const int KC = (int)wp.KC;
  if (N % KC) return fail(GGNN_EUNSUP, "rows not divisible into weight-gradient chunks");
  a.KC = KC;
  a.nchunks = (int)(N / KC);
  {
    Prof p(K_WGRAD, s);
    if (KC % 64 != 0 || wp.KCt % 64 != 0) hipLaunchKernelGGL((k_wgrad<32, WP>), dim3(wgs), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_wgrad<64, WP>), dim3(wgs), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_wgrad_reduce<128>, dim3(tiles * 16), dim3(256), 0, s, a);
  }
  LAUNCHCHK();
  return GGNN_OK;
}

#include "generic_path.h"

int pack_impl(const Cfg& c, void* pack, const unsigned char* chocc, const float* W, const float* beta,
              const float* Wg, const float* bg, const float* Wc, const float* bc, hipStream_t s) {
  const PackL L = pack_layout(c);
  const int H = c.H;
  PackJobs a;
  memset(&a, 0, sizeof(a));
  a.dr = c.edrop;
  a.chocc = chocc;
  int nb = 0;
  auto flush = [&]() {
    if (!a.count) return;
    a.blk_begin[a.count] = nb;
    Prof p(K_PACK, s);
    if (c.prec != PREC_BF16) hipLaunchKernelGGL(k_pack_multi<true>, dim3(nb), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_pack_multi<false>, dim3(nb), dim3(256), 0, s, a);
    a.count = 0;
    nb = 0;
  };
  auto job = [&](const float* S, int ldS, long sS, int K, int N, int trans, void* out, long sO, long lo, int batch,
                 int t, int drop, int f8 = 0) {
    if (a.count == PACK_MAXJ) flush();  // (long T under edge dropout)
    PackJob& J = a.j[a.count];
    J.S = S; J.out = (u16*)out; J.sS = sS; J.sO = sO; J.lo_off = lo;
    J.total = (long)batch * (N / 32) * (K / 16) * 64;
    J.ldS = ldS; J.K = K; J.N = N; J.trans = trans; J.t = t; J.drop = drop; J.copy = 0; J.f8 = f8;
    a.blk_begin[a.count++] = nb;
    nb += (int)((J.total + 255) / 256);
  };
  auto copy = [&](const float* S, float* out, long n, int mode = 1, int t = 0, int drop = 0, uint32_t* bits = nullptr) {
    if (a.count == PACK_MAXJ) flush();
    PackJob& J = a.j[a.count];
    // mode 2: 16-byte pieces when H % 4 == 0 and both ends are 16-byte aligned
    // (masked: one thread per 32-row block of 4 columns); else one thread per
    // element, or per 32-row block of a column when masked (a partial last
    // quad when H % 4 != 0)
    const int vec = mode == 2 && H % 4 == 0 && !(((uintptr_t)S | (uintptr_t)out) & 15);
    const long w32 = (H + 31) / 32;
    if (mode == 2 && vec) n = drop ? (long)c.C * w32 * (H / 4) : n / 4;
    else if (mode == 2 && drop) n = (long)c.C * w32 * H;
    J.S = S; J.out = (u16*)out; J.total = n; J.copy = mode; J.K = H; J.t = t; J.drop = drop; J.trans = vec;
    J.bits = drop ? bits : nullptr;
    a.blk_begin[a.count++] = nb;
    nb += (int)((n + 255) / 256);
  };
  if (L.fast) {
    for (int t = 0; t < (c.ed ? c.T : 1); ++t) {  // one masked copy per timestep under edge dropout
      job(W, H, (long)H * H, H, H, 0, P<u16>(pack, L.wf(t)), (long)H * H, L.loW, c.C, t, c.ed);  // MT: Bmat = W_c
      // dh: Bmat = W_c^T; fp32-parity mode: fp8 correction fragments (k_prop_bwd, mfma_f8corr)
      job(W, H, (long)H * H, H, H, 1, P<u16>(pack, L.wt(t)), (long)H * H, L.loW, c.C, t, c.ed, prop_f8(c));
    }
    job(Wg, 2 * H, 0, 2 * H, 2 * H, 0, P<u16>(pack, L.Wg), 0, L.loWg, 1, 0, 0);
    // k_gru_bwd's W^T packs: fp32-parity mode: fp8 lo fragments (gb_f8_product)
    const int gf8 = c.prec == PREC_SPLIT ? 2 : 0;
    job(Wg, 2 * H, 0, 2 * H, 2 * H, 1, P<u16>(pack, L.WgT), 0, L.loWg, 1, 0, 0, gf8);
    job(Wc, H, 0, 2 * H, H, 0, P<u16>(pack, L.Wc), 0, L.loWc, 1, 0, 0);   // Bmat = Wc   [2H][H]
    job(Wc, H, 0, H, 2 * H, 1, P<u16>(pack, L.WcT), 0, L.loWc, 1, 0, 0, gf8);  // Bmat = Wc^T [H][2H]
  }
  copy((c.flags & GGNN_USE_EDGE_BIAS) ? beta : nullptr, P<float>(pack, L.beta), (long)c.C * H);
  copy(bg, P<float>(pack, L.bg), 2L * H);
  copy(bc, P<float>(pack, L.bc), (long)H);
  // the general path's fp32 operands (generic_path.h), also in a pack made for
  // the specialised kernels: a pack is made with b = v = 1 dims and may serve a
  // later general-path batch (v > 128).  Measured cost at config 3: 3.5 MB of
  // copies, the whole pack launch 0.013 ms per step (profiles/r03b_bench.json)
  for (int t = 0; t < (c.ed ? c.T : 1); ++t)
    copy(W, P<float>(pack, L.gw(t)), (long)c.C * H * H, 2, t, c.ed, c.ed ? P<uint32_t>(pack, L.gb(t)) : nullptr);
  copy(Wg, P<float>(pack, L.gWg), 4L * H * H);
  copy(Wc, P<float>(pack, L.gWc), 2L * H * H);
  flush();
  LAUNCHCHK();
  return GGNN_OK;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {
#ifdef GGNN_TS
int ggnn_dbg_ts(void* host) { return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ts), sizeof(g_ts)); }
int ggnn_dbg_clk(void* host) { return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_clk), sizeof(g_clk)); }
int ggnn_dbg_ts_clear(void) {
  static unsigned long long zero[sizeof(g_ts) / 8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ts), zero, sizeof(g_ts));
}
#endif

int ggnn_version(void) { return 4; }
const char* ggnn_last_error(void) { return g_err.c_str(); }

const char* ggnn_kernel_kind_name(int kind) {
  return (kind >= 0 && kind < GGNN_NUM_KERNEL_KINDS) ? kKindNames[kind] : "";
}

int ggnn_profile_begin(int max_launches) {
  if (max_launches < 1) return fail(GGNN_EINVAL, "profile_begin: max_launches < 1");
  for (hipEvent_t e : g_prof.ev)
    if (e) (void)hipEventDestroy(e);
  g_prof.ev.assign(2 * (size_t)max_launches, nullptr);
  g_prof.kind.assign(max_launches, 0);
  for (auto& e : g_prof.ev) HIPCHK(hipEventCreate(&e));
  g_prof.cap = max_launches;
  g_prof.used = 0;
  g_prof.on = true;
  return GGNN_OK;
}

int ggnn_profile_end(double* total_ms, int* launches) {
  if (!g_prof.on) return fail(GGNN_EINVAL, "profile_end without profile_begin");
  g_prof.on = false;
  for (int k = 0; k < GGNN_NUM_KERNEL_KINDS; ++k) {
    if (total_ms) total_ms[k] = 0.0;
    if (launches) launches[k] = 0;
  }
  for (int i = 0; i < g_prof.used; ++i) {
    HIPCHK(hipEventSynchronize(g_prof.ev[2 * i + 1]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
    if (total_ms) total_ms[g_prof.kind[i]] += ms;
    if (launches) launches[g_prof.kind[i]] += 1;
  }
  const int overflow = g_prof.used >= g_prof.cap;
  g_prof.used = 0;
  return overflow ? fail(GGNN_EINVAL, "profile buffer full: raise max_launches") : GGNN_OK;
}

int ggnn_check_dims(const ggnn_dims* d) {
  Cfg c;
  return make_cfg(d, &c);
}

int ggnn_workspace_bytes(const ggnn_dims* d, int training, size_t* bytes) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = c.generic ? gen_ws_layout(c, training != 0).total : ws_layout(c, training != 0).total;
  return GGNN_OK;
}

int ggnn_adjacency_bytes(const ggnn_dims* d, size_t* bytes) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = c.generic ? gen_adj_layout(c).total : adj_layout(c).total;
  return GGNN_OK;
}

int ggnn_weight_pack_bytes(const ggnn_dims* d, size_t* bytes) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!bytes) return fail(GGNN_EINVAL, "bytes is NULL");
  *bytes = pack_layout(c).total;
  return GGNN_OK;
}


int ggnn_pack_weights(const ggnn_dims* d, void* pack, const float* W, const float* beta, const float* Wg,
                      const float* bg, const float* Wc, const float* bc, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!pack || !W || !Wg || !bg || !Wc || !bc) return fail(GGNN_EINVAL, "pack_weights: NULL pointer");
  if ((c.flags & GGNN_USE_EDGE_BIAS) && !beta)
    return fail(GGNN_EINVAL, "pack_weights: edge_biases NULL with USE_EDGE_BIAS");
  return pack_impl(c, pack, nullptr, W, beta, Wg, bg, Wc, bc, (hipStream_t)stream);
}

int ggnn_pack_weights_batch(const ggnn_dims* d, void* pack, const void* adj, const float* W, const float* beta,
                            const float* Wg, const float* bg, const float* Wc, const float* bc,
                            ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!pack || !adj || !W || !Wg || !bg || !Wc || !bc) return fail(GGNN_EINVAL, "pack_weights_batch: NULL pointer");
  if ((c.flags & GGNN_USE_EDGE_BIAS) && !beta)
    return fail(GGNN_EINVAL, "pack_weights_batch: edge_biases NULL with USE_EDGE_BIAS");
  hipStream_t s = (hipStream_t)stream;
  const unsigned char* chocc = nullptr;
  if (c.generic && c.ed && !(c.flags & GGNN_DENSE_CHANNELS)) {
    // the general path reads W_c only for channels with an edge in the batch
    // (the tiles / pairs of the others are empty): mask only those copies.
    // Not under GGNN_DENSE_CHANNELS: there every (graph, channel) tile is run
    // (k_gen_lists counts them all), so M = h W_c reads every channel's copy
    // and an unwritten one would enter the products as 0 * (stale bits)
    const PackL L = pack_layout(c);
    unsigned char* oc = P<unsigned char>(pack, L.chocc);
    Prof p(K_PACK, s);
    hipLaunchKernelGGL(k_chan_any, dim3((c.C + 255) / 256), dim3(256), 0, s,
                       P<const unsigned char>(adj, gen_adj_layout(c).occ), c.b, c.C, oc);
    chocc = oc;
  }
  return pack_impl(c, pack, chocc, W, beta, Wg, bg, Wc, bc, s);
}

int ggnn_dropout_mask(const ggnn_dims* d, int kind, int t, uint8_t* mask, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!mask) return fail(GGNN_EINVAL, "dropout_mask: NULL pointer");
  if (kind != 0 && kind != 1) return fail(GGNN_EINVAL, "dropout_mask: kind must be 0 (edge) or 1 (state)");
  if (t < 0 || t >= c.T) return fail(GGNN_EINVAL, "dropout_mask: t outside [0, T)");
  hipStream_t s = (hipStream_t)stream;
  const long total = kind == 0 ? (long)c.C * c.H * c.H : (long)c.b * c.vin * c.H;
  hipLaunchKernelGGL(k_dropout_mask, dim3(grid1d(total)), dim3(256), 0, s, kind, c.C, c.H, c.b, c.vin, t,
                     kind == 0 ? c.edrop : c.sdrop, mask);
  LAUNCHCHK();
  return GGNN_OK;
}

static int adam_impl(const ggnn_adam_tensor* tensors, int count, float learning_rate, float beta1, float beta2,
                     float epsilon, float clip_norm, int64_t step, const int64_t* step_dev, float grad_scale,
                     float* scratch, ggnn_stream_t stream) {
  if (!tensors || !scratch) return fail(GGNN_EINVAL, "adam_step: NULL pointer");
  if (count < 1 || count > GGNN_OPT_MAXT)
    return fail(GGNN_EINVAL, "adam_step: count must be in 1.." + std::to_string(GGNN_OPT_MAXT));
  if (!step_dev && step < 1) return fail(GGNN_EINVAL, "adam_step: step counts from 1");
  if (!(clip_norm > 0.f)) return fail(GGNN_EINVAL, "adam_step: clip_norm must be > 0");
  OptArgs a;
  memset(&a, 0, sizeof(a));
  a.count = count;
  long off = 0;
  for (int i = 0; i < count; ++i) {
    const ggnn_adam_tensor& t = tensors[i];
    if (!t.param || !t.grad || !t.m || !t.v || t.n < 1) return fail(GGNN_EINVAL, "adam_step: bad tensor entry");
    a.t[i] = OptTensor{t.param, t.grad, t.m, t.v, (long)t.n, t.sqnorm};
    a.begin[i] = off;
    off += t.n;
  }
  a.begin[count] = off;
  // TF1 Adam folds both bias corrections into the step size
  if (step_dev) {
    a.step = step_dev;
    a.lr = learning_rate;
  } else {
    const double b1t = std::pow((double)beta1, (double)step), b2t = std::pow((double)beta2, (double)step);
    a.lr_t = (float)(learning_rate * std::sqrt(1.0 - b2t) / (1.0 - b1t));
  }
  a.gscale = grad_scale;
  a.clip = clip_norm;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = epsilon;
  hipStream_t s = (hipStream_t)stream;
  Prof p(K_OPT, s);
  long maxn = 1;
  for (int i = 0; i < count; ++i) maxn = std::max<long>(maxn, a.t[i].n);
  // scratch holds count * OPT_BLOCKS per-block partial norms
  const dim3 grid((unsigned)std::min<long>(GGNN_ADAM_SCRATCH_PER_TENSOR, (maxn + OPT_THREADS - 1) / OPT_THREADS),
                  (unsigned)count);
  hipLaunchKernelGGL(k_opt_sqnorm, grid, dim3(OPT_THREADS), 0, s, a, scratch);
  hipLaunchKernelGGL(k_opt_adam, grid, dim3(OPT_THREADS), 0, s, a, (const float*)scratch);
  LAUNCHCHK();
  return GGNN_OK;
}
int ggnn_adam_step(const ggnn_adam_tensor* tensors, int count, float learning_rate, float beta1, float beta2,
                   float epsilon, float clip_norm, int64_t step, float grad_scale, float* scratch,
                   ggnn_stream_t stream) {
  return adam_impl(tensors, count, learning_rate, beta1, beta2, epsilon, clip_norm, step, nullptr, grad_scale, scratch,
                   stream);
}
int ggnn_adam_step_dev(const ggnn_adam_tensor* tensors, int count, float learning_rate, float beta1, float beta2,
                       float epsilon, float clip_norm, const int64_t* step, float grad_scale, float* scratch,
                       ggnn_stream_t stream) {
  if (!step) return fail(GGNN_EINVAL, "adam_step_dev: NULL step");
  return adam_impl(tensors, count, learning_rate, beta1, beta2, epsilon, clip_norm, 0, step, grad_scale, scratch,
                   stream);
}

int ggnn_set_adjacency_edges(const ggnn_dims* d, void* adj, const int32_t* edges, const int32_t* graph_offsets,
                             int64_t num_edges, int num_edge_types, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!adj || !graph_offsets || (num_edges > 0 && !edges)) return fail(GGNN_EINVAL, "set_adjacency_edges: NULL pointer");
  if (num_edge_types < 1 || 2 * num_edge_types != c.C)
    return fail(GGNN_EINVAL, "set_adjacency_edges: C must equal 2 * num_edge_types");
  if (num_edges < 0) return fail(GGNN_EINVAL, "set_adjacency_edges: num_edges < 0");
  if (c.sparse && num_edges > (int64_t)c.b * c.vin)
    return fail(GGNN_EUNSUP, "set_adjacency_edges: GGNN_SPARSE_PAIRS needs num_edges <= b * v");
  hipStream_t s = (hipStream_t)stream;
  if (c.generic) {
    if (int e2 = gen_set_adjacency_edges(c, adj, edges, graph_offsets, num_edges, num_edge_types, s)) return e2;
    LAUNCHCHK();
    return GGNN_OK;
  }
  const AdjL L = adj_layout(c);
  const size_t tiles = (size_t)c.b * c.C;
  Prof p(K_ADJ, s);
  fill_async(P<u16>(adj, L.Ab), 0, tiles * c.V * c.V * 2, s);
  fill_async(P<u16>(adj, L.AbT), 0, tiles * c.V * c.V * 2, s);
  const int grid = grid1d(std::max<int64_t>(num_edges, 1));
#define ADJ_EDGES(VV, F)                                                                                         \
  do {                                                                                                           \
    if (num_edges > 0)                                                                                           \
      hipLaunchKernelGGL((k_adj_from_edges<VV, F>), dim3(grid), dim3(256), 0, s, edges, graph_offsets, c.b,      \
                         c.vin, num_edge_types, P<u16>(adj, L.Ab), P<u16>(adj, L.AbT));                           \
    hipLaunchKernelGGL((k_adj_deg<VV, F>), dim3((unsigned)tiles), dim3(VV), 0, s, P<const u16>(adj, L.Ab),        \
                       P<u16>(adj, L.deg));                                                                      \
    hipLaunchKernelGGL(k_chan_list<VV>, dim3(c.b), dim3(256), 0, s, P<const u16>(adj, L.deg), c.C,               \
                       P<int>(adj, L.chl), P<int>(adj, L.chl_all), P<unsigned char>(adj, L.occ));                \
    hipLaunchKernelGGL(k_chan_graphs, dim3(c.C), dim3(64), 0, s, P<const unsigned char>(adj, L.occ), c.b, c.C,   \
                       P<int>(adj, L.cgl));                                                                      \
  } while (0)
  const bool f16 = c.prec != PREC_BF16;
  if (c.V == 32) { if (f16) ADJ_EDGES(32, true); else ADJ_EDGES(32, false); }
  else if (c.V == 64) { if (f16) ADJ_EDGES(64, true); else ADJ_EDGES(64, false); }
  else { if (f16) ADJ_EDGES(128, true); else ADJ_EDGES(128, false); }
#undef ADJ_EDGES
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_set_adjacency(const ggnn_dims* d, void* adj, const float* A, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!adj || !A) return fail(GGNN_EINVAL, "set_adjacency: NULL pointer");
  if (c.sparse) return fail(GGNN_EINVAL, "set_adjacency: GGNN_SPARSE_PAIRS batches are staged by set_adjacency_edges");
  hipStream_t s = (hipStream_t)stream;
  if (c.generic) {
    if (int e2 = gen_set_adjacency(c, adj, A, s)) return e2;
    LAUNCHCHK();
    return GGNN_OK;
  }
  const AdjL L = adj_layout(c);
  const dim3 grid((unsigned)(c.b * c.C));
  Prof p(K_ADJ, s);
#define PREP_ADJ(VV, F)                                                                                       \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_prep_adj<VV, F>), grid, dim3(256), 0, s, A, c.vin, P<u16>(adj, L.Ab),                 \
                       P<u16>(adj, L.AbT), P<u16>(adj, L.deg));                                               \
    hipLaunchKernelGGL(k_chan_list<VV>, dim3(c.b), dim3(256), 0, s, P<const u16>(adj, L.deg), c.C,             \
                       P<int>(adj, L.chl), P<int>(adj, L.chl_all), P<unsigned char>(adj, L.occ));              \
    hipLaunchKernelGGL(k_chan_graphs, dim3(c.C), dim3(64), 0, s, P<const unsigned char>(adj, L.occ), c.b, c.C, \
                       P<int>(adj, L.cgl));                                                                    \
  } while (0)
  if (c.prec != PREC_BF16) {
    if (c.V == 32) PREP_ADJ(32, true);
    else if (c.V == 64) PREP_ADJ(64, true);
    else PREP_ADJ(128, true);
  } else {
    if (c.V == 32) PREP_ADJ(32, false);
    else if (c.V == 64) PREP_ADJ(64, false);
    else PREP_ADJ(128, false);
  }
#undef PREP_ADJ
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_forward(const ggnn_dims* d, const void* pack, const void* adj, void* ws, int training, const float* h0,
                 float* hT, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!pack || !adj || !ws || !h0 || !hT) return fail(GGNN_EINVAL, "forward: NULL pointer");
  hipStream_t s = (hipStream_t)stream;
  if (c.generic) {
    void* adjw = const_cast<void*>(adj);  // (the channel lists are rebuilt per call)
    switch (c.prec) {
      case PREC_SPLIT: return gen_forward<PREC_SPLIT>(c, pack, adjw, ws, training != 0, h0, hT, s);
      case PREC_F16: return gen_forward<PREC_F16>(c, pack, adjw, ws, training != 0, h0, hT, s);
      default: return gen_forward<PREC_BF16>(c, pack, adjw, ws, training != 0, h0, hT, s);
    }
  }
  switch (c.prec) {
    case PREC_SPLIT: return forward_impl<PREC_SPLIT>(c, pack, adj, ws, training != 0, h0, hT, s);
    case PREC_F16: return forward_impl<PREC_F16>(c, pack, adj, ws, training != 0, h0, hT, s);
    default: return forward_impl<PREC_BF16>(c, pack, adj, ws, training != 0, h0, hT, s);
  }
}

int ggnn_backward(const ggnn_dims* d, const void* pack, const void* adj, void* ws, const float* dhT, float* dh0,
                  float* dW, float* dbeta, float* dWg, float* dbg, float* dWc, float* dbc, ggnn_stream_t stream) {
  Cfg c;
  int e = make_cfg(d, &c);
  if (e) return e;
  if (!pack || !adj || !ws || !dhT || !dh0 || !dW || !dWg || !dbg || !dWc || !dbc)
    return fail(GGNN_EINVAL, "backward: NULL pointer");
  if ((c.flags & GGNN_USE_EDGE_BIAS) && !dbeta)
    return fail(GGNN_EINVAL, "backward: d_edge_biases NULL with USE_EDGE_BIAS");
  hipStream_t s = (hipStream_t)stream;
  if (c.generic) {
    void* adjw = const_cast<void*>(adj);
    switch (c.prec) {
      case PREC_SPLIT: return gen_backward<PREC_SPLIT>(c, pack, adjw, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
      case PREC_F16: return gen_backward<PREC_F16>(c, pack, adjw, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
      default: return gen_backward<PREC_BF16>(c, pack, adjw, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
    }
  }
  switch (c.prec) {
    case PREC_SPLIT: return backward_impl<PREC_SPLIT>(c, pack, adj, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
    case PREC_F16: return backward_impl<PREC_F16>(c, pack, adj, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
    default: return backward_impl<PREC_BF16>(c, pack, adj, ws, dhT, dh0, dW, dbeta, dWg, dbg, dWc, dbc, s);
  }
}

// ---- test / tuning hook: D[M][N] = A[M][K] B[K][N] (row-major fp32) through
// k_gemm in the precision of d->flags (the general path's product kernel)
int ggnn_dbg_gemm(const ggnn_dims* d, int M, int N, int K, const float* A, const float* B, float* D,
                  ggnn_stream_t stream) {
  Cfg c;
  if (int e = make_cfg(d, &c)) return e;
  if (!A || !B || !D || M < 1 || N < 1 || K < 1) return fail(GGNN_EINVAL, "dbg_gemm: bad arguments");
  GemmArgs a = gg_args();
  a.A = A; a.sAm = K; a.sAk = 1;
  a.B = B; a.sBk = N; a.sBn = 1;
  a.D = D; a.sDm = N; a.sDn = 1;
  a.M = M; a.N = N; a.K = K;
  hipStream_t s = (hipStream_t)stream;
  switch (c.prec) {
    case PREC_SPLIT: return gg_launch<PREC_SPLIT>(a, false, true, false, K_PROP_FWD, s);
    case PREC_F16: return gg_launch<PREC_F16>(a, false, true, false, K_PROP_FWD, s);
    default: return gg_launch<PREC_BF16>(a, false, true, false, K_PROP_FWD, s);
  }
}

int ggnn_dbg_gemm_ex(const ggnn_dims* d, int M, int N, int K, const void* A, int a_layout, const float* B,
                     int b_layout, float* D, int kernel, ggnn_stream_t stream) {
  Cfg c;
  if (int e = make_cfg(d, &c)) return e;
  if (!A || !B || !D || M < 1 || N < 1 || K < 1 || a_layout < 0 || a_layout > 2 || b_layout < 0 || b_layout > 1 ||
      kernel < 0 || kernel > 5)
    return fail(GGNN_EINVAL, "dbg_gemm_ex: bad arguments");
  GemmArgs a = gg_args();
  const bool akc = a_layout != 1, a16 = a_layout == 2, bkc = b_layout == 1;
  a.A = A;
  if (akc) { a.sAm = K; a.sAk = 1; } else { a.sAm = 1; a.sAk = M; }
  a.B = B;
  if (bkc) { a.sBn = K; a.sBk = 1; } else { a.sBn = 1; a.sBk = N; }
  a.D = D; a.sDm = N; a.sDn = 1;
  a.M = M; a.N = N; a.K = K;
  if (kernel >= 2 && !ring_ok(a, a16, akc, bkc)) return fail(GGNN_EINVAL, "dbg_gemm_ex: operands not ring-aligned");
  hipStream_t s = (hipStream_t)stream;
  g_gemm_force = kernel;
  int e;
  switch (c.prec) {
    case PREC_SPLIT: e = gg_launch<PREC_SPLIT>(a, a16, akc, bkc, K_PROP_FWD, s); break;
    case PREC_F16: e = gg_launch<PREC_F16>(a, a16, akc, bkc, K_PROP_FWD, s); break;
    default: e = gg_launch<PREC_BF16>(a, a16, akc, bkc, K_PROP_FWD, s); break;
  }
  g_gemm_force = 0;
  return e;
}

// ---- embedding front-end and output heads (k_head.h)
static int plain_dims(const ggnn_dims* d, const char* what) {
  if (!d) return fail(GGNN_EINVAL, std::string(what) + ": dims is NULL");
  if (d->b < 1 || d->v < 1 || d->h < 1) return fail(GGNN_EINVAL, std::string(what) + ": b, v, h must be >= 1");
  return GGNN_OK;
}
static int check_keep(float keep, const char* what) {
  if (!(keep > 0.f && keep <= 1.f)) return fail(GGNN_EINVAL, std::string(what) + ": keep must lie in (0, 1]");
  return GGNN_OK;
}
static int emb_args(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, int ncols, float keep, uint64_t seed,
                    EmbArgs* a, const char* what) {
  if (int e = plain_dims(d, what)) return e;
  if (int e = check_keep(keep, what)) return e;
  if (!segs || nseg < 1 || nseg > GGNN_EMBED_MAX_SEGMENTS)
    return fail(GGNN_EINVAL, std::string(what) + ": 1.." + std::to_string(GGNN_EMBED_MAX_SEGMENTS) + " segments");
  memset(a, 0, sizeof(*a));
  int off = 0;
  for (int i = 0; i < nseg; ++i) {
    const ggnn_embed_segment& g = segs[i];
    if (!g.table || g.rows < 1 || g.width < 1 || g.column < 0 || g.column >= ncols)
      return fail(GGNN_EINVAL, std::string(what) + ": bad segment " + std::to_string(i));
    a->s[i] = EmbSeg{g.table, (long)g.rows, g.width, g.column, off};
    off += g.width;
  }
  // the reference pads the concat up to hidden_size with tf.pad, which fails
  // for a negative pad (80+50+100+80 = 310 > 256)
  if (off > d->h)
    return fail(GGNN_EINVAL, std::string(what) + ": embedding widths sum to " + std::to_string(off) + " > hidden " +
                                 std::to_string(d->h) + " (negative pad)");
  a->nseg = nseg;
  a->ncols = ncols;
  a->H = d->h;
  a->rows = (long)d->b * d->v;
  if ((d->flags & GGNN_SEED_DEVICE) && !seed && keep < 1.0f)
    return fail(GGNN_EINVAL, std::string(what) + ": GGNN_SEED_DEVICE needs a device seed address");
  a->dr = make_drop(keep, seed, (d->flags & GGNN_SEED_DEVICE) != 0);
  return GGNN_OK;
}

int ggnn_embed_forward(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, const int32_t* word_inputs,
                       int ncols, float keep, uint64_t seed, float* h0, ggnn_stream_t stream) {
  EmbArgs a;
  if (int e = emb_args(d, segs, nseg, ncols, keep, seed, &a, "embed_forward")) return e;
  if (!word_inputs || !h0) return fail(GGNN_EINVAL, "embed_forward: NULL pointer");
  hipStream_t s = (hipStream_t)stream;
  Prof p(K_HEADS, s);
  hipLaunchKernelGGL(k_embed_fwd, dim3(grid1d((a.rows + 3) / 4 * a.H)), dim3(256), 0, s, a, word_inputs, h0);
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_embed_backward(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, const int32_t* word_inputs,
                        int ncols, float keep, uint64_t seed, const float* dh0, const float* dh0_add,
                        float* lookup_sqnorm, ggnn_stream_t stream) {
  EmbArgs a;
  if (int e = emb_args(d, segs, nseg, ncols, keep, seed, &a, "embed_backward")) return e;
  if (!word_inputs || !dh0 || !lookup_sqnorm) return fail(GGNN_EINVAL, "embed_backward: NULL pointer");
  EmbGrad gd;
  memset(&gd, 0, sizeof(gd));
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < nseg; ++i) {
    if (!segs[i].d_table) return fail(GGNN_EINVAL, "embed_backward: NULL d_table");
    gd.dtable[i] = segs[i].d_table;
    // a table looked up by several segments has ONE gradient (the reference's
    // IndexedSlices concatenate both lookups' rows): its squared norm goes to
    // the slot of the first segment with that d_table
    gd.sqslot[i] = i;
    for (int j = 0; j < i; ++j)
      if (segs[j].d_table == segs[i].d_table) { gd.sqslot[i] = j; break; }
  }
  Prof p(K_HEADS, s);
  {
    Zeroer z(s);
    for (int i = 0; i < nseg; ++i) z.add(segs[i].d_table, (long)segs[i].rows * segs[i].width);
    z.add(lookup_sqnorm, nseg);
  }
  hipLaunchKernelGGL(k_embed_bwd, dim3(std::min(grid1d((a.rows + 3) / 4 * a.H), 4096)), dim3(256), 0, s, a, gd, word_inputs,
                     dh0, dh0_add, lookup_sqnorm);
  LAUNCHCHK();
  return GGNN_OK;
}

// ---- deterministic embedding backward (fixed-point accumulation, k_head.h)
namespace {
struct EmbWsL {
  size_t acc[GGNN_EMBED_MAX_SEGMENTS], own[GGNN_EMBED_MAX_SEGMENTS], sqp, total;
};
// one accumulator and owner-slot region per segment (segments sharing a
// d_table use the first one's at call time)
int emb_ws_layout(const ggnn_embed_segment* segs, int nseg, EmbWsL* L, const char* what) {
  if (!segs || nseg < 1 || nseg > GGNN_EMBED_MAX_SEGMENTS)
    return fail(GGNN_EINVAL, std::string(what) + ": 1.." + std::to_string(GGNN_EMBED_MAX_SEGMENTS) + " segments");
  size_t o = 0;
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].rows < 1 || segs[i].width < 1) return fail(GGNN_EINVAL, std::string(what) + ": bad segment");
    L->acc[i] = o; o += al((size_t)segs[i].rows * segs[i].width * 8);
    L->own[i] = o; o += al((size_t)segs[i].rows * 4);
  }
  L->sqp = o; o += al((size_t)EMB_SQ_BLOCKS * EMB_MAXSEG * 4);
  L->total = o;
  return GGNN_OK;
}
}  // namespace

int ggnn_embed_workspace_bytes(const ggnn_embed_segment* segs, int nseg, size_t* bytes) {
  EmbWsL L;
  if (int e = emb_ws_layout(segs, nseg, &L, "embed_workspace_bytes")) return e;
  if (!bytes) return fail(GGNN_EINVAL, "embed_workspace_bytes: NULL pointer");
  *bytes = L.total;
  return GGNN_OK;
}

int ggnn_embed_backward_ws(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, const int32_t* word_inputs,
                           int ncols, float keep, uint64_t seed, const float* dh0, const float* dh0_add,
                           float* lookup_sqnorm, void* ws, ggnn_stream_t stream) {
  EmbArgs a;
  if (int e = emb_args(d, segs, nseg, ncols, keep, seed, &a, "embed_backward_ws")) return e;
  EmbWsL L;
  if (int e = emb_ws_layout(segs, nseg, &L, "embed_backward_ws")) return e;
  if (!word_inputs || !dh0 || !lookup_sqnorm || !ws) return fail(GGNN_EINVAL, "embed_backward_ws: NULL pointer");
  EmbGrad gd;
  EmbAcc ea;
  memset(&gd, 0, sizeof(gd));
  memset(&ea, 0, sizeof(ea));
  for (int i = 0; i < nseg; ++i) {
    gd.dtable[i] = segs[i].d_table;
    if (!segs[i].d_table) continue;  // no gradient for this segment (its sq slot: 0)
    // segments sharing a d_table (btb: the loc table, word_inputs columns 0
    // and 3) accumulate in the first one's region; its squared norm slot too
    int u = i;
    for (int j = 0; j < i; ++j)
      if (segs[j].d_table == segs[i].d_table) { u = j; break; }
    if (segs[u].rows != segs[i].rows || segs[u].width != segs[i].width)
      return fail(GGNN_EINVAL, "embed_backward_ws: segments sharing a d_table disagree on its shape");
    gd.sqslot[i] = u;
    ea.acc[i] = P<long long>(ws, L.acc[u]);
    ea.own[i] = P<int>(ws, L.own[u]);
  }
  if (a.rows * nseg > 0x7fffffffL / 64 || a.rows >= (1L << 27))
    return fail(GGNN_EINVAL, "embed_backward_ws: too many lookup rows");
  hipStream_t s = (hipStream_t)stream;
  Prof p(K_HEADS, s);
  {
    Zeroer z(s);
    for (int i = 0; i < nseg; ++i)
      if (segs[i].d_table) z.add(segs[i].d_table, (long)segs[i].rows * segs[i].width);
  }
  const int nblk = std::min(grid1d((a.rows + 3) / 4 * a.H), EMB_SQ_BLOCKS);
  float* sqp = P<float>(ws, L.sqp);
  hipLaunchKernelGGL(k_embed_bwd_det, dim3(nblk), dim3(256), 0, s, a, ea, word_inputs, dh0, dh0_add, sqp);
  const long waves = a.rows * nseg;
  hipLaunchKernelGGL(k_embed_fin, dim3((unsigned)((waves + 3) / 4 + 1)), dim3(256), 0, s, a, ea, gd, word_inputs, sqp,
                     nblk, lookup_sqnorm);
  LAUNCHCHK();
  return GGNN_OK;
}

int ggnn_embed_lookup_rows(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, int seg,
                           const int32_t* word_inputs, int ncols, float keep, uint64_t seed, const float* dh0,
                           const float* dh0_add, float* rows, int32_t* ids, int64_t cap, ggnn_stream_t stream) {
  EmbArgs a;
  if (int e = emb_args(d, segs, nseg, ncols, keep, seed, &a, "embed_lookup_rows")) return e;
  if (seg < 0 || seg >= nseg) return fail(GGNN_EINVAL, "embed_lookup_rows: segment out of range");
  if (!word_inputs || !dh0 || !rows || !ids) return fail(GGNN_EINVAL, "embed_lookup_rows: NULL pointer");
  if (cap < a.rows) return fail(GGNN_EINVAL, "embed_lookup_rows: cap < b * v lookup rows");
  hipStream_t s = (hipStream_t)stream;
  Prof p(K_HEADS, s);
  hipLaunchKernelGGL(k_embed_rows, dim3(grid1d(cap * segs[seg].width)), dim3(256), 0, s, a, seg, word_inputs, dh0,
                     dh0_add, rows, ids, (long)cap);
  LAUNCHCHK();
  return GGNN_OK;
}

namespace {
// All heads side by side: head i owns columns [off[i], off[i] + o_i) of the
// concatenated operands (width Ot, each head padded to a multiple of 4 with
// zeros), so a head set costs ONE logits, one d[hT | h0] and one dW product
// (two heads one by one: 3 + 3 launches with 128-column tiles over o = 150 and
// 46, and a read-modify-write pass over dX for the second head).
constexpr int HEAD_LP = 2048;  // loss partials per head (one per softmax block)
struct HeadL {
  int off[GGNN_MAX_HEADS], Ot;
  size_t W, Sx, bias, Z, dZ, dW, lp, slab, dbp, sums, total;
};
// the heads' dW product: split-K over node rows, chunks of KC rows
long head_dw_kc(long rows) { return std::max<long>(256, ((rows + 47) / 48 + 31) & ~31L); }
constexpr int HEAD_DZ_BLOCKS = 256;  // k_head_dz blocks (at most): one bias partial row each
int head_layout(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, HeadL* L, const char* what) {
  if (int e = plain_dims(d, what)) return e;
  if (!heads || nheads < 1 || nheads > GGNN_MAX_HEADS)
    return fail(GGNN_EINVAL, std::string(what) + ": 1.." + std::to_string(GGNN_MAX_HEADS) + " heads");
  const size_t rows = (size_t)d->b * d->v, K = 2 * (size_t)d->h;
  int Ot = 0;
  for (int i = 0; i < nheads; ++i) {
    if (heads[i].o < 1 || heads[i].o > HEAD_MAXO || !heads[i].weight || !heads[i].bias)
      return fail(GGNN_EINVAL, std::string(what) + ": bad head " + std::to_string(i));
    L->off[i] = Ot;
    Ot += (heads[i].o + 3) & ~3;
  }
  L->Ot = Ot;
  size_t o = 0;
  L->W = o;    o += al(K * Ot * 4);     // dropped weights W * mask / keep
  L->Sx = o;   o += al(K * Ot * 4);     // mask / keep
  L->bias = o; o += al((size_t)Ot * 4);
  L->Z = o;    o += al(rows * Ot * 4);  // logits
  L->dZ = o;   o += al(rows * Ot * 4);
  L->dW = o;   o += al(K * Ot * 4);
  L->lp = o;   o += al((size_t)nheads * HEAD_LP * 4);
  // deterministic reductions: the dW product's split-K slab, the bias
  // partials of k_head_dz (one row per block) and k_sum_rows' chunk sums
  const long kc = head_dw_kc((long)rows);
  L->slab = o; o += al((size_t)((rows + kc - 1) / kc) * K * Ot * 4);
  L->dbp = o;  o += al((size_t)HEAD_DZ_BLOCKS * Ot * 4);
  L->sums = o; o += al((size_t)SUM_RCS * Ot * 4);
  L->total = o;
  return GGNN_OK;
}
}  // namespace

int ggnn_heads_workspace_bytes(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, size_t* bytes) {
  HeadL L;
  if (int e = head_layout(d, heads, nheads, &L, "heads_workspace_bytes")) return e;
  if (!bytes) return fail(GGNN_EINVAL, "heads_workspace_bytes: NULL pointer");
  *bytes = L.total;
  return GGNN_OK;
}

// target_num: a host value, or (tn_dev) read from device memory by the kernels
static int heads_forward_impl(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                              const float* h0, float keep, uint64_t seed, float target_num, const float* tn_dev,
                              float* loss, void* ws, ggnn_stream_t stream) {
  HeadL L;
  if (int e = head_layout(d, heads, nheads, &L, "heads_forward")) return e;
  if (int e = check_keep(keep, "heads_forward")) return e;
  if (!hT || !h0 || !ws) return fail(GGNN_EINVAL, "heads_forward: NULL pointer");
  if (!tn_dev && !(target_num > 0.f)) return fail(GGNN_EINVAL, "heads_forward: target_num must be > 0");
  if ((d->flags & GGNN_SEED_DEVICE) && !seed && keep < 1.0f)
    return fail(GGNN_EINVAL, "heads_forward: GGNN_SEED_DEVICE needs a device seed address");
  for (int i = 0; i < nheads; ++i)
    if (!heads[i].probs) return fail(GGNN_EINVAL, "heads_forward: NULL probs");
  hipStream_t s = (hipStream_t)stream;
  const int H = d->h, K = 2 * H, Ot = L.Ot;
  const long rows = (long)d->b * d->v;
  const Drop dr = make_drop(keep, seed, (d->flags & GGNN_SEED_DEVICE) != 0);
  Prof p(K_HEADS, s);
  float* W = P<float>(ws, L.W);
  float* Z = P<float>(ws, L.Z);
  for (int i = 0; i < nheads; ++i) {
    const int o = heads[i].o, op = (o + 3) & ~3;
    hipLaunchKernelGGL(k_head_wdrop, dim3(grid1d((long)K * op)), dim3(256), 0, s, heads[i].weight, heads[i].bias, K, o,
                       op, Ot, L.off[i], i, dr, W, P<float>(ws, L.Sx), P<float>(ws, L.bias));
  }
  // z = [hT | h0] W + b for every head at once, on MFMA (split f16 limbs, fp32
  // accumulation): two terms, one per half of the concatenation
  GemmArgs q = gg_args();
  q.A = hT; q.A2 = h0; q.sAm = H; q.sAk = 1;
  q.B = W; q.sBq = (long)H * Ot; q.sBk = Ot; q.sBn = 1;
  q.D = Z; q.sDm = Ot; q.sDn = 1;
  q.bias = P<const float>(ws, L.bias);
  q.nterm = 2; q.M = (int)rows; q.N = Ot; q.K = H;
  if (int e = gg_launch<PREC_SPLIT>(q, false, true, false, -1, s)) return e;
  const unsigned nb = (unsigned)std::min<long>(HEAD_LP, (rows + 7) / 8);
  for (int i = 0; i < nheads; ++i) {
    const ggnn_output_head& hd = heads[i];
    const int o = hd.o;
    const float* y = loss ? hd.labels : (const float*)nullptr;
    float* lp = P<float>(ws, L.lp) + (long)i * HEAD_LP;
#define HSM(NI_)                                                                                                  \
  hipLaunchKernelGGL(k_head_softmax<NI_>, dim3(nb), dim3(256), 0, s, Z + L.off[i], Ot, hd.probs, y, rows, o, \
                     tn_dev ? 1.0f : 1.0f / target_num, tn_dev, lp)
    if (o <= 64) HSM(1);
    else if (o <= 128) HSM(2);
    else if (o <= 256) HSM(4);
    else HSM(HEAD_MAXO / 64);
#undef HSM
    if (loss) hipLaunchKernelGGL(k_head_loss, dim3(1), dim3(256), 0, s, lp, (int)nb, loss + i);
  }
  LAUNCHCHK();
  return GGNN_OK;
}
int ggnn_heads_forward(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT, const float* h0,
                       float keep, uint64_t seed, float target_num, float* loss, void* ws, ggnn_stream_t stream) {
  return heads_forward_impl(d, heads, nheads, hT, h0, keep, seed, target_num, nullptr, loss, ws, stream);
}
int ggnn_heads_forward_dev(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                           const float* h0, float keep, uint64_t seed, const float* target_num, float* loss, void* ws,
                           ggnn_stream_t stream) {
  if (!target_num) return fail(GGNN_EINVAL, "heads_forward_dev: NULL target_num");
  return heads_forward_impl(d, heads, nheads, hT, h0, keep, seed, 0.f, target_num, loss, ws, stream);
}

static int heads_backward_impl(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                               const float* h0, float target_num, const float* tn_dev, const float* d_loss, void* ws,
                               float* dhT, float* dh0, ggnn_stream_t stream) {
  HeadL L;
  if (int e = head_layout(d, heads, nheads, &L, "heads_backward")) return e;
  if (!hT || !h0 || !ws || !dhT || !dh0) return fail(GGNN_EINVAL, "heads_backward: NULL pointer");
  if (!tn_dev && !(target_num > 0.f)) return fail(GGNN_EINVAL, "heads_backward: target_num must be > 0");
  hipStream_t s = (hipStream_t)stream;
  const int H = d->h, K = 2 * H, Ot = L.Ot;
  const long rows = (long)d->b * d->v;
  for (int i = 0; i < nheads; ++i)
    if (!heads[i].labels || !heads[i].probs || !heads[i].d_weight || !heads[i].d_bias)
      return fail(GGNN_EINVAL, "heads_backward: head needs labels, probs, d_weight, d_bias");
  Prof p(K_HEADS, s);
  float* dZ = P<float>(ws, L.dZ);
  float* dW = P<float>(ws, L.dW);
  float* dbp = P<float>(ws, L.dbp);
  // (every bias and dW element is stored once by the fixed-order sums below)
  const int nbz = (int)std::min<long>(HEAD_DZ_BLOCKS, (rows + 15) / 16);
  SumPlan sp(P<float>(ws, L.sums));
  for (int i = 0; i < nheads; ++i) {
    const ggnn_output_head& hd = heads[i];
    const int o = hd.o, op = (o + 3) & ~3;
    // bias: one column-partial row per block (dbp[block][off + j]), summed in block order
#define HDZ(NI_)                                                                                                  \
  hipLaunchKernelGGL(k_head_dz<NI_>, dim3((unsigned)nbz), dim3(256), 0, s, hd.probs, hd.labels, rows, o, op,    \
                     tn_dev ? 1.0f : 1.0f / target_num, tn_dev, d_loss, dZ + L.off[i], Ot, dbp + L.off[i], Ot)
    if (op <= 64) HDZ(1);
    else if (op <= 128) HDZ(2);
    else if (op <= 256) HDZ(4);
    else HDZ(HEAD_MAXO / 64);
#undef HDZ
    sp.add(dbp + L.off[i], 1, nbz, 0, Ot, o, o, 0, hd.d_bias, hd.d_bias, o);
  }
  if (int e = sp.launch(s)) return e;
  // dZ ~ 1/target_num per element: carried as S*dZ (S an exact power of two
  // <= target_num) so its f16 limbs stay normal; alpha = 1/S undoes it
  // (tn_dev: the GEMMs resolve S from the device value, GemmArgs::snum)
  const float S = tn_dev ? 2.0f : tnum_scale(target_num);
  const float* W = P<const float>(ws, L.W);
  // (hidden a multiple of 64: each product in one launch with the output /
  // operand split at H; otherwise one launch per half)
  const bool one = H % 64 == 0;
  const long KC = head_dw_kc(rows);
  for (int half = 0; half < (one ? 1 : 2); ++half) {
    // [dhT | dh0] = dZ W^T  (B(k=j, n=c) = W[c][j]; K = Ot: padding columns are zeros)
    GemmArgs q = gg_args();
    q.A = dZ; q.sAm = Ot; q.sAk = 1; q.scA = S; q.alpha = 1.0f / S; q.snum = tn_dev; q.sdev = 1;
    q.B = W + (long)half * H * Ot; q.sBk = 1; q.sBn = Ot;
    q.D = half ? dh0 : dhT; q.sDm = H; q.sDn = 1;
    q.M = (int)rows; q.N = one ? 2 * H : H; q.K = Ot;
    if (one) { q.D2 = dh0; q.Nsplit = H; }
    if (int e = gg_launch<PREC_SPLIT>(q, false, true, true, -1, s)) return e;
    // dW[rows of the half] += (mask / keep) * ([hT | h0]^T dZ): split-K over node rows, atomics
    GemmArgs w = gg_args();
    w.A = half ? h0 : hT; w.sAp = KC * H; w.sAm = 1; w.sAk = H;
    w.B = dZ; w.sBp = KC * Ot; w.sBk = Ot; w.sBn = 1; w.scB = S; w.alpha = 1.0f / S; w.snum = tn_dev; w.sdev = 2;
    w.D = dW + (long)half * H * Ot; w.sDm = Ot; w.sDn = 1; w.mode = GG_ATOMIC;
    w.E = P<const float>(ws, L.Sx) + (long)half * H * Ot;
    w.Z = (int)((rows + KC - 1) / KC); w.M = one ? 2 * H : H; w.N = Ot; w.K = (int)KC; w.Ktot = rows; w.sKp = KC;
    if (one) { w.Am2 = h0; w.Msplit = H; }
    // the row chunks' partials in a slab, summed in chunk order (deterministic)
    w.slab = P<float>(ws, L.slab); w.sSlab = (long)w.M * Ot;
    if (int e = gg_launch<PREC_SPLIT>(w, false, false, false, -1, s)) return e;
    slab_reduce(w, 1, w.Z, nullptr, 0, 0, 0, s);
  }
  for (int i = 0; i < nheads; ++i)
    hipLaunchKernelGGL(k_head_dw_out, dim3(grid1d((long)K * heads[i].o)), dim3(256), 0, s, dW + L.off[i], Ot, K,
                       heads[i].o, heads[i].d_weight);
  LAUNCHCHK();
  return GGNN_OK;
}
int ggnn_heads_backward(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT, const float* h0,
                        float target_num, const float* d_loss, void* ws, float* dhT, float* dh0,
                        ggnn_stream_t stream) {
  return heads_backward_impl(d, heads, nheads, hT, h0, target_num, nullptr, d_loss, ws, dhT, dh0, stream);
}
int ggnn_heads_backward_dev(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                            const float* h0, const float* target_num, const float* d_loss, void* ws, float* dhT,
                            float* dh0, ggnn_stream_t stream) {
  if (!target_num) return fail(GGNN_EINVAL, "heads_backward_dev: NULL target_num");
  return heads_backward_impl(d, heads, nheads, hT, h0, 0.f, target_num, d_loss, ws, dhT, dh0, stream);
}

}  // extern "C"
