// PyTorch bindings of the gfx950 kernels (module _C). Every op takes preallocated tensors (no allocation on the
// hot path, graph-capture safe) and launches on the current HIP stream of the tensors' device.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/launch.h"

namespace {

using OptT = std::optional<at::Tensor>;

void check(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

template <typename T>
T* ptr(const at::Tensor& t, const char* name) {
  check(t, name);
  return reinterpret_cast<T*>(t.data_ptr());
}

template <typename T>
T* optr(const OptT& t, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
  return ptr<T>(*t, name);
}

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void ok(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " failed (code " + std::to_string(rc) + ")");
}

InXform xf(const OptT& ab, int C, int relu) { return InXform{optr<const float>(ab, "ab"), C, relu}; }

// fused BN-node gradient epilogue arguments (launch.h BnNodeEpi); node_y = None -> off
BnNodeEpi node_epi_args(const OptT& node_y, const OptT& node_ab, const OptT& node_sums, int reps, int relu,
                        int64_t out_numel, int C) {
  BnNodeEpi e{};
  if (!node_y) return e;
  TORCH_CHECK(node_ab && node_sums, "node epilogue: node_ab and node_sums are required with node_y");
  e.y = ptr<const bf16_t>(*node_y, "node_y");
  e.ab = ptr<const float>(*node_ab, "node_ab");
  e.sums = ptr<float>(*node_sums, "node_sums");
  e.reps = reps < 1 ? 1 : reps;
  e.relu = relu;
  TORCH_CHECK(node_y->numel() == out_numel, "node epilogue: node_y must have the output's shape");
  TORCH_CHECK(node_ab->numel() >= 4 * C && node_sums->numel() >= (int64_t)e.reps * 2 * C, "node epilogue sizes");
  return e;
}

// BN finalize arguments of a consumer that computes its input's coefficients itself (launch.h BnStatsIn)
BnStatsIn stats_in(const OptT& stats, const OptT& gamma, const OptT& beta, double count, double eps, int C,
                   const OptT& ab) {
  BnStatsIn f{};
  if (!stats) return f;
  TORCH_CHECK(gamma && beta && ab && count > 0 && stats->numel() >= (int64_t)STAT_REPLICAS * 2 * C &&
              gamma->numel() >= C && beta->numel() >= C && ab->numel() >= 4 * C,
              "consumer-side BN finalize: needs stats, gamma, beta and the ab destination");
  f.stats = ptr<const float>(*stats, "fin_stats");
  f.gamma = ptr<const float>(*gamma, "fin_gamma");
  f.beta = ptr<const float>(*beta, "fin_beta");
  f.count = (float)count;
  f.eps = (float)eps;
  return f;
}

BnBwdApplyParams bba_params(at::Tensor g, at::Tensor y, at::Tensor ab, at::Tensor sums, at::Tensor dy, OptT dgamma,
                            OptT dbeta, int M, int C, int sum_reps) {
  BnBwdApplyParams p{};
  p.sum_reps = sum_reps < 1 ? 1 : sum_reps;
  TORCH_CHECK(sums.numel() >= (int64_t)p.sum_reps * 2 * C, "bn_bwd_apply: sums size");
  p.g = ptr<const bf16_t>(g, "g");
  p.y = ptr<const bf16_t>(y, "y");
  p.ab = ptr<const float>(ab, "ab");
  p.sums = ptr<const float>(sums, "sums");
  p.dy = ptr<bf16_t>(dy, "dy");
  p.dgamma = optr<float>(dgamma, "dgamma");
  p.dbeta = optr<float>(dbeta, "dbeta");
  p.M = M; p.C = C;
  TORCH_CHECK(g.numel() == (int64_t)M * C && y.numel() == g.numel() && dy.numel() == g.numel(), "bn_bwd_apply sizes");
  return p;
}

OptT opt_at(const py::tuple& t, int i) { return t[i].is_none() ? OptT() : OptT(t[i].cast<at::Tensor>()); }

// side jobs of a streaming 1x1 dgrad (launch.h SideJob), as tuples of the standalone ops' arguments:
//   side_bba  = (g, y, ab, sums, dy, dgamma, dbeta, M, C, reps)               (bn_bwd_apply)
//   side_pool = (src, argmax, v, ab, out, sums, B, H, W, C, reps)            (node_bwd, GM_MAXPOOL routing)
SideJob side_job(const py::object& side_bba, const py::object& side_pool) {
  SideJob j{};
  TORCH_CHECK(side_bba.is_none() || side_pool.is_none(), "conv_igemm: one side job at most");
  if (!side_bba.is_none()) {
    const py::tuple t = side_bba.cast<py::tuple>();
    TORCH_CHECK(t.size() == 10, "side_bba: (g, y, ab, sums, dy, dgamma, dbeta, M, C, reps)");
    j.kind = SIDE_BBA;
    j.bba = bba_params(t[0].cast<at::Tensor>(), t[1].cast<at::Tensor>(), t[2].cast<at::Tensor>(),
                       t[3].cast<at::Tensor>(), t[4].cast<at::Tensor>(), opt_at(t, 5), opt_at(t, 6), t[7].cast<int>(),
                       t[8].cast<int>(), t[9].cast<int>());
  } else if (!side_pool.is_none()) {
    const py::tuple t = side_pool.cast<py::tuple>();
    TORCH_CHECK(t.size() == 11, "side_pool: (src, argmax, v, ab, out, sums, B, H, W, C, reps)");
    const at::Tensor src = t[0].cast<at::Tensor>(), am = t[1].cast<at::Tensor>(), v = t[2].cast<at::Tensor>();
    const at::Tensor ab = t[3].cast<at::Tensor>(), out = t[4].cast<at::Tensor>(), sums = t[5].cast<at::Tensor>();
    NodeBwdParams& q = j.pool;
    q.src[0] = GradSrc{ptr<const bf16_t>(src, "src"), GM_MAXPOOL, 0};
    q.src[1] = GradSrc{nullptr, GM_NONE, 0};
    q.argmax = ptr<const uint8_t>(am, "argmax");
    q.v = ptr<const bf16_t>(v, "v");
    q.ab = ptr<const float>(ab, "ab");
    q.out = ptr<bf16_t>(out, "out");
    q.sums = ptr<float>(sums, "sums");
    q.B = t[6].cast<int>(); q.H = t[7].cast<int>(); q.W = t[8].cast<int>(); q.C = t[9].cast<int>();
    q.sum_reps = t[10].cast<int>() < 1 ? 1 : t[10].cast<int>();
    const int64_t n = (int64_t)q.B * q.H * q.W * q.C, half = (int64_t)q.B * ((q.H + 1) / 2) * ((q.W + 1) / 2) * q.C;
    TORCH_CHECK(v.numel() == n && out.numel() == n && src.numel() == half && am.numel() == half &&
                ab.numel() >= 4 * q.C && sums.numel() >= (int64_t)q.sum_reps * 2 * q.C, "side_pool sizes");
    j.kind = SIDE_POOL;
  }
  return j;
}

void conv_igemm_op(at::Tensor x, at::Tensor wt, OptT bias, at::Tensor y, OptT stats, OptT ab, int relu, int B,
                   int Hin, int Win, int Cin, int up_in, int Ho, int Wo, int N, int ks, int stride, int pad_t,
                   int pad_l, OptT ws, int algo, OptT node_y, OptT node_ab, OptT node_sums, int node_reps,
                   int node_relu, int join_mode, OptT join_y, OptT join_ab, OptT join_out, OptT join_argmax,
                   int join_H, int join_W, OptT bwd_y, OptT bwd_ab, OptT bwd_sums, int bwd_reps, OptT bwd_dx, OptT bwd_dgamma,
                   OptT bwd_dbeta, OptT pj_v, OptT pj_add, OptT pj_out, OptT pj_sy, OptT pj_sab, OptT pj_sums,
                   int pj_reps, OptT jfin_stats, OptT jfin_gamma, OptT jfin_beta, double jfin_count,
                   double jfin_eps, OptT xfin_stats, OptT xfin_gamma, OptT xfin_beta, double xfin_count,
                   double xfin_eps, OptT sum2x2, py::object side_bba, py::object side_pool, OptT wt8,
                   OptT ws8) {
  ConvParams p{};
  p.algo = algo;
  p.x = ptr<const bf16_t>(x, "x");
  p.wt = ptr<const bf16_t>(wt, "wt");
  p.bias = optr<const float>(bias, "bias");
  p.y = ptr<bf16_t>(y, "y");
  p.stats = optr<float>(stats, "stats");
  p.xf = xf(ab, Cin, relu);
  p.xfin = stats_in(xfin_stats, xfin_gamma, xfin_beta, xfin_count, xfin_eps, Cin, ab);
  p.B = B; p.Hin = Hin; p.Win = Win; p.Cin = Cin; p.up_in = up_in;
  p.Ho = Ho; p.Wo = Wo; p.N = N; p.ks = ks; p.stride = stride; p.pad_t = pad_t; p.pad_l = pad_l;
  p.M = B * Ho * Wo;
  p.K = ks * ks * Cin;
  p.ws = optr<float>(ws, "ws");
  p.ws_elems = p.ws ? ws->numel() : 0;
  TORCH_CHECK(x.numel() == (int64_t)B * Hin * Win * Cin, "conv_igemm: x size");
  TORCH_CHECK(wt.numel() >= (int64_t)N * p.K, "conv_igemm: wt size");
  TORCH_CHECK(y.numel() == (int64_t)p.M * N, "conv_igemm: y size");
  TORCH_CHECK(!p.stats || stats->numel() >= (int64_t)STAT_REPLICAS * 2 * N, "conv_igemm: stats size");
  p.node = node_epi_args(node_y, node_ab, node_sums, node_reps, node_relu, y.numel(), N);
  TORCH_CHECK(!p.node.y || (!p.stats && !p.bias), "conv_igemm: the node epilogue excludes stats and bias");
  if (join_mode) {
    TORCH_CHECK(join_mode >= JOIN_POOL && join_mode <= JOIN_ADD_UP && join_y && join_ab && join_out,
                "conv_igemm: join needs join_y, join_ab, join_out");
    TORCH_CHECK(ks == 1 && !p.stats && !p.node.y && N % 8 == 0, "conv_igemm: joins are for 1x1 convs without stats");
    const int64_t yn = (int64_t)B * join_H * join_W * N;
    TORCH_CHECK(join_y->numel() == yn && join_ab->numel() >= 4 * N, "conv_igemm: join_y / join_ab size");
    if (join_mode == JOIN_POOL) {
      TORCH_CHECK(Ho == (join_H + 1) / 2 && Wo == (join_W + 1) / 2 && join_argmax &&
                  join_out->numel() == (int64_t)p.M * N && join_argmax->numel() == (int64_t)p.M * N,
                  "conv_igemm: pool join shapes");
    } else {
      const int u = join_mode == JOIN_ADD_UP ? 2 : 1;
      TORCH_CHECK(join_H == u * Ho && join_W == u * Wo && join_out->numel() == yn, "conv_igemm: add join shapes");
    }
    p.join.mode = join_mode;
    p.join.y = ptr<const bf16_t>(*join_y, "join_y");
    p.join.ab = ptr<const float>(*join_ab, "join_ab");
    p.join.out = ptr<bf16_t>(*join_out, "join_out");
    p.join.argmax = optr<uint8_t>(join_argmax, "join_argmax");
    p.join.H = join_H;
    p.join.W = join_W;
    p.join.fin = stats_in(jfin_stats, jfin_gamma, jfin_beta, jfin_count, jfin_eps, N, join_ab);
  }
  if (bwd_y) {                      // BN-backward apply folded into the operand load (common.h BnBwdIn)
    TORCH_CHECK(bwd_ab && bwd_sums && bwd_dx, "conv_igemm: bwd_y needs bwd_ab, bwd_sums, bwd_dx");
    TORCH_CHECK(!ab && !relu && !up_in && !join_mode && Cin <= BNB_MAX_C && bwd_reps >= 1 &&
                bwd_reps <= BNB_MAX_REPS, "conv_igemm: the folded BN backward excludes ab / relu / up_in / join");
    TORCH_CHECK(bwd_y->numel() == x.numel() && bwd_dx->numel() == x.numel() && bwd_ab->numel() >= 4 * Cin &&
                bwd_sums->numel() >= (int64_t)bwd_reps * 2 * Cin, "conv_igemm: bwd tensor sizes");
    TORCH_CHECK((!bwd_dgamma || bwd_dgamma->numel() >= Cin) && (!bwd_dbeta || bwd_dbeta->numel() >= Cin),
                "conv_igemm: bwd_dgamma / bwd_dbeta sizes");
    p.bwd.y = ptr<const bf16_t>(*bwd_y, "bwd_y");
    p.bwd.ab = ptr<const float>(*bwd_ab, "bwd_ab");
    p.bwd.sums = ptr<const float>(*bwd_sums, "bwd_sums");
    p.bwd.reps = bwd_reps;
    p.bwd.invM = 1.f / (float)((int64_t)B * Hin * Win);
    p.bwd.dx = ptr<bf16_t>(*bwd_dx, "bwd_dx");
    p.bwd.dgamma = optr<float>(bwd_dgamma, "bwd_dgamma");
    p.bwd.dbeta = optr<float>(bwd_dbeta, "bwd_dbeta");
  }
  if (pj_v) {                       // decoder node join at half resolution (launch.h PoolJoinEpi)
    TORCH_CHECK(pj_out && ks == 3 && stride == 1 && Ho % 2 == 0 && Wo % 2 == 0 && !p.stats && !p.bias &&
                !p.node.y && !join_mode, "conv_igemm: pj_* is a 3x3 dgrad epilogue (no stats / bias / node / join)");
    const int64_t hn = (int64_t)B * (Ho / 2) * (Wo / 2) * N;
    TORCH_CHECK(pj_v->numel() == hn && pj_out->numel() == hn && (!pj_add || pj_add->numel() == hn) &&
                (!pj_sy || (pj_sy->numel() == hn && pj_sab && pj_sab->numel() >= 4 * N && pj_sums &&
                            pj_sums->numel() >= (int64_t)(pj_reps < 1 ? 1 : pj_reps) * 2 * N)),
                "conv_igemm: pj tensor sizes");
    p.pj.v = ptr<const bf16_t>(*pj_v, "pj_v");
    p.pj.add = optr<const bf16_t>(pj_add, "pj_add");
    p.pj.out = ptr<bf16_t>(*pj_out, "pj_out");
    p.pj.sy = optr<const bf16_t>(pj_sy, "pj_sy");
    p.pj.sab = optr<const float>(pj_sab, "pj_sab");
    p.pj.sums = p.pj.sy ? ptr<float>(*pj_sums, "pj_sums") : nullptr;
    p.pj.reps = pj_reps < 1 ? 1 : pj_reps;
  }
  if (sum2x2) {                     // x = 2x2-block sums of sum2x2, formed on load and stored into x
    TORCH_CHECK(sum2x2->numel() == 4 * x.numel() && ks == 1 && stride == 1 && !up_in && !ab && !relu && !bwd_y &&
                !p.bias && !p.stats && !node_y && !join_mode && !pj_v, "conv_igemm: sum2x2 is a plain 1x1 dgrad input");
    p.sum2x2 = ptr<const bf16_t>(*sum2x2, "sum2x2");
  }
  p.side = side_job(side_bba, side_pool);
  if (wt8) {                        // block-scaled fp8 operands of a 3x3 conv (fp8.hip)
    TORCH_CHECK(ws8 && wt8->scalar_type() == at::kByte && ws8->scalar_type() == at::kByte &&
                wt8->numel() >= (int64_t)N * p.K && ws8->numel() >= (int64_t)N * (p.K / 32),
                "conv_igemm: wt8 [N][K] e4m3 bytes with ws8 [N][K/32] e8m0 scales");
    p.wt8 = ptr<const uint8_t>(*wt8, "wt8");
    p.ws8 = ptr<const uint8_t>(*ws8, "ws8");
    TORCH_CHECK(conv3x3_f8_supported(p), "conv_igemm: fp8 operands need a 3x3 / stride-1 conv, Cin % 32 == 0, "
                "Cin <= 256, N % 32 == 0, no BN-backward fold");
  }
  ok(conv_igemm(p, stream()), "conv_igemm");
}

int conv_splits_op(int B, int Ho, int Wo, int N, int ks, int stride, int pad, int Cin) {
  ConvParams p{};
  p.B = B; p.Ho = Ho; p.Wo = Wo; p.N = N; p.ks = ks; p.stride = stride; p.pad_t = pad; p.pad_l = pad; p.Cin = Cin;
  p.M = B * Ho * Wo;
  p.K = ks * ks * Cin;
  return conv_igemm_splits(p);
}

WgradParams wgrad_params(at::Tensor x, at::Tensor dy, at::Tensor dw, OptT ab, int relu, int B, int Hin, int Win,
                         int Cin, int up_in, int Ho, int Wo, int N, int ks, int stride, int pad_t, int pad_l,
                         int dst_mode, int m_chunk, int algo, int slabs) {
  WgradParams p{};
  p.x = ptr<const bf16_t>(x, "x");
  p.dy = ptr<const bf16_t>(dy, "dy");
  p.dw = ptr<float>(dw, "dw");
  p.xf = xf(ab, Cin, relu);
  p.B = B; p.Hin = Hin; p.Win = Win; p.Cin = Cin; p.up_in = up_in;
  p.Ho = Ho; p.Wo = Wo; p.N = N; p.ks = ks; p.stride = stride; p.pad_t = pad_t; p.pad_l = pad_l;
  p.M = B * Ho * Wo;
  p.K = ks * ks * Cin;
  p.dst_mode = dst_mode;
  p.m_chunk = m_chunk;
  p.algo = algo;
  p.slabs = slabs;
  TORCH_CHECK(slabs <= 0 || slabs == conv_wgrad_slabs(p), "conv_wgrad: slab rows != conv_wgrad_slabs()");
  TORCH_CHECK(slabs <= 0 || !conv_wgrad_plain_slabs(p) || dw.numel() == (int64_t)slabs * p.K * N,
              "conv_wgrad: a plain-stored slab must be exactly rows * K * N");
  TORCH_CHECK(x.numel() == (int64_t)B * Hin * Win * Cin, "conv_wgrad: x size");
  TORCH_CHECK(dy.numel() == (int64_t)p.M * N, "conv_wgrad: dy size");
  TORCH_CHECK(dw.numel() >= (int64_t)(slabs > 0 ? slabs : 1) * p.K * N, "conv_wgrad: dw size");
  return p;
}

void conv_wgrad_op(at::Tensor x, at::Tensor dy, at::Tensor dw, OptT ab, int relu, int B, int Hin, int Win, int Cin,
                   int up_in, int Ho, int Wo, int N, int ks, int stride, int pad_t, int pad_l, int dst_mode,
                   int m_chunk, int algo, int slabs) {
  const WgradParams p = wgrad_params(x, dy, dw, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t, pad_l,
                                     dst_mode, m_chunk, algo, slabs);
  ok(conv_wgrad(p, stream()), "conv_wgrad");
}

// calls: a list of conv_wgrad argument tuples (x, dy, dw, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride,
// pad_t, pad_l, dst_mode, m_chunk, algo, slabs) -> one batch (3x3 halo wgrads grouped into shared launches)
// fused pointwise backward (pw_bwd.hip): g, y [B,H,W,K]; d, dd [B,H,W,N]; w [N*K] packed PK_PW_DGRAD; dw replica
// rows [replicas][N*K] (x2 int64 in the deterministic mode); the BN rows / sums of the BN that y feeds
bool pw_bwd_supported_op(int B, int H, int W, int K, int N) {
  PwBwdParams p{};
  p.M = B * H * W;
  p.K = K;
  p.N = N;
  p.replicas = 1;
  p.bwd.reps = 1;
  return pw_bwd_supported(p);
}

void pw_bwd_op(torch::Tensor g, torch::Tensor y, torch::Tensor ab, torch::Tensor sums, int reps, torch::Tensor w,
               torch::Tensor d, torch::Tensor dd, torch::Tensor dw, int replicas, OptT dgamma, OptT dbeta, int B,
               int H, int W, int K, int N) {
  const int64_t M = (int64_t)B * H * W;
  TORCH_CHECK(g.numel() == M * K && y.numel() == M * K && d.numel() == M * N && dd.numel() == M * N &&
              w.numel() >= (int64_t)N * K && ab.numel() >= 4 * K && sums.numel() >= (int64_t)reps * 2 * K &&
              dw.numel() >= (int64_t)replicas * N * K * (cfl_det_host() ? 2 : 1), "pw_bwd: tensor sizes");
  PwBwdParams p{};
  p.g = ptr<const bf16_t>(g, "g");
  p.y = ptr<const bf16_t>(y, "y");
  p.d = ptr<const bf16_t>(d, "d");
  p.w = ptr<const bf16_t>(w, "w");
  p.dd = ptr<bf16_t>(dd, "dd");
  p.dw = ptr<float>(dw, "dw");
  p.bwd.y = p.y;
  p.bwd.ab = ptr<const float>(ab, "ab");
  p.bwd.sums = ptr<const float>(sums, "sums");
  p.bwd.reps = reps;
  p.bwd.invM = 1.f / (float)M;
  p.bwd.dgamma = optr<float>(dgamma, "dgamma");
  p.bwd.dbeta = optr<float>(dbeta, "dbeta");
  p.M = (int)M;
  p.K = K;
  p.N = N;
  p.replicas = replicas;
  TORCH_CHECK(pw_bwd_supported(p), "pw_bwd: unsupported shape");
  ok(pw_bwd(p, stream()), "pw_bwd");
}

void conv_wgrad_batch_op(py::list calls) {
  std::vector<WgradParams> ps;
  for (auto h : calls) {
    auto t = h.cast<py::tuple>();
    TORCH_CHECK(t.size() == 21, "conv_wgrad_batch: each call needs the 21 conv_wgrad arguments");
    OptT ab = t[3].is_none() ? OptT() : OptT(t[3].cast<at::Tensor>());
    ps.push_back(wgrad_params(t[0].cast<at::Tensor>(), t[1].cast<at::Tensor>(), t[2].cast<at::Tensor>(), ab,
                              t[4].cast<int>(), t[5].cast<int>(), t[6].cast<int>(), t[7].cast<int>(),
                              t[8].cast<int>(), t[9].cast<int>(), t[10].cast<int>(), t[11].cast<int>(),
                              t[12].cast<int>(), t[13].cast<int>(), t[14].cast<int>(), t[15].cast<int>(),
                              t[16].cast<int>(), t[17].cast<int>(), t[18].cast<int>(), t[19].cast<int>(),
                              t[20].cast<int>()));
  }
  ok(conv_wgrad_batch(ps.data(), (int)ps.size(), stream()), "conv_wgrad_batch");
}

// (slab rows, rows are plain-stored (sum without re-zeroing) rather than atomic replicas)
std::tuple<int, bool> conv_wgrad_slabs_op(int B, int Hin, int Win, int Cin, int up_in, int Ho, int Wo, int N, int ks,
                                          int stride, int pad_t, int pad_l, int algo) {
  WgradParams p{};
  p.B = B; p.Hin = Hin; p.Win = Win; p.Cin = Cin; p.up_in = up_in;
  p.Ho = Ho; p.Wo = Wo; p.N = N; p.ks = ks; p.stride = stride; p.pad_t = pad_t; p.pad_l = pad_l;
  p.M = B * Ho * Wo;
  p.K = ks * ks * Cin;
  p.algo = algo;
  return {conv_wgrad_slabs(p), conv_wgrad_plain_slabs(p)};
}

SepParams sepp(at::Tensor x, OptT ab, int relu, at::Tensor wdw, at::Tensor wpw, OptT bias, at::Tensor d, at::Tensor y,
               OptT stats, int B, int H, int W, int K, int N, OptT xfin_stats, OptT xfin_gamma, OptT xfin_beta,
               double xfin_count, double xfin_eps) {
  SepParams p{};
  p.x = ptr<const bf16_t>(x, "x");
  p.xf = xf(ab, K, relu);
  p.xfin = stats_in(xfin_stats, xfin_gamma, xfin_beta, xfin_count, xfin_eps, K, ab);
  p.wdw = ptr<const float>(wdw, "wdw");
  p.wpw = ptr<const bf16_t>(wpw, "wpw");
  p.bias = optr<const float>(bias, "bias");
  p.d = ptr<bf16_t>(d, "d");
  p.y = ptr<bf16_t>(y, "y");
  p.stats = optr<float>(stats, "stats");
  p.B = B; p.H = H; p.W = W; p.K = K; p.N = N;
  const int64_t px = (int64_t)B * H * W;
  TORCH_CHECK(x.numel() == px * K && d.numel() == px * K && y.numel() == px * N && wdw.numel() == 9 * K &&
              wpw.numel() == (int64_t)K * N && (!bias || bias->numel() == N) &&
              (!stats || stats->numel() >= (int64_t)STAT_REPLICAS * 2 * N) && (!ab || ab->numel() >= 2 * K),
              "sep_fwd sizes");
  return p;
}

bool sep_fwd_supported_op(int B, int H, int W, int K, int N) {
  SepParams p{};
  p.B = B; p.H = H; p.W = W; p.K = K; p.N = N;
  return sep_fwd_supported(p);
}

void sep_fwd_op(at::Tensor x, OptT ab, int relu, at::Tensor wdw, at::Tensor wpw, OptT bias, at::Tensor d, at::Tensor y,
                OptT stats, int B, int H, int W, int K, int N, OptT xfin_stats, OptT xfin_gamma, OptT xfin_beta,
                double xfin_count, double xfin_eps) {
  ok(sep_fwd(sepp(x, ab, relu, wdw, wpw, bias, d, y, stats, B, H, W, K, N, xfin_stats, xfin_gamma, xfin_beta,
                  xfin_count, xfin_eps), stream()), "sep_fwd");
}

DwParams dwp(int B, int H, int W, int C) {
  DwParams p{};
  p.B = B; p.H = H; p.W = W; p.C = C;
  return p;
}

void dw_fwd_op(at::Tensor x, at::Tensor w, at::Tensor y, OptT ab, int relu, int B, int H, int W, int C, int algo,
               OptT xfin_stats, OptT xfin_gamma, OptT xfin_beta, double xfin_count, double xfin_eps) {
  DwParams p = dwp(B, H, W, C);
  p.algo = algo;
  p.x = ptr<const bf16_t>(x, "x");
  p.w = ptr<const float>(w, "w");
  p.y = ptr<bf16_t>(y, "y");
  p.xf = xf(ab, C, relu);
  p.xfin = stats_in(xfin_stats, xfin_gamma, xfin_beta, xfin_count, xfin_eps, C, ab);
  TORCH_CHECK(x.numel() == (int64_t)B * H * W * C && y.numel() == x.numel() && w.numel() == 9 * C, "dw_fwd sizes");
  ok(dw_fwd(p, stream()), "dw_fwd");
}

void dw_dgrad_op(at::Tensor dy, at::Tensor w, at::Tensor dx, int B, int H, int W, int C, int algo, OptT node_y,
                 OptT node_ab, OptT node_sums, int node_reps, int node_relu) {
  DwParams p = dwp(B, H, W, C);
  p.algo = algo;
  p.node = node_epi_args(node_y, node_ab, node_sums, node_reps, node_relu, dx.numel(), C);
  p.dy = ptr<const bf16_t>(dy, "dy");
  p.w = ptr<const float>(w, "w");
  p.y = ptr<bf16_t>(dx, "dx");
  TORCH_CHECK(dy.numel() == (int64_t)B * H * W * C && dx.numel() == dy.numel() && w.numel() == 9 * C, "dw_dgrad sizes");
  ok(dw_dgrad(p, stream()), "dw_dgrad");
}

DwParams dw_wgrad_params(at::Tensor x, at::Tensor dy, at::Tensor dw, OptT ab, int relu, int B, int H, int W, int C,
                         int replicas, int algo) {
  DwParams p = dwp(B, H, W, C);
  p.algo = algo;
  p.x = ptr<const bf16_t>(x, "x");
  p.dy = ptr<const bf16_t>(dy, "dy");
  p.dw = ptr<float>(dw, "dw");
  p.xf = xf(ab, C, relu);
  p.replicas = replicas < 1 ? 1 : replicas;
  TORCH_CHECK(x.numel() == (int64_t)B * H * W * C && dy.numel() == x.numel() &&
                  dw.numel() == (cfl_det_host() ? 2 : 1) * (int64_t)p.replicas * 9 * C, "dw_wgrad sizes");
  return p;
}

void dw_wgrad_op(at::Tensor x, at::Tensor dy, at::Tensor dw, OptT ab, int relu, int B, int H, int W, int C,
                 int replicas, int algo) {
  ok(dw_wgrad(dw_wgrad_params(x, dy, dw, ab, relu, B, H, W, C, replicas, algo), stream()), "dw_wgrad");
}

void dw_bwd_op(at::Tensor x, OptT ab, int relu, at::Tensor dy, at::Tensor w, at::Tensor dx, at::Tensor dw,
               int replicas, int B, int H, int W, int C, int algo, OptT node_y, OptT node_ab, OptT node_sums,
               int node_reps, int node_relu, OptT add_half, int mask_x) {
  DwParams p = dw_wgrad_params(x, dy, dw, ab, relu, B, H, W, C, replicas, algo);
  p.w = ptr<const float>(w, "w");
  p.y = ptr<bf16_t>(dx, "dx");
  p.node = node_epi_args(node_y, node_ab, node_sums, node_reps, node_relu, dx.numel(), C);
  p.add_half = optr<const bf16_t>(add_half, "add_half");
  p.mask_x = mask_x;
  TORCH_CHECK(!p.add_half || add_half->numel() == (int64_t)B * ((H + 1) / 2) * ((W + 1) / 2) * C,
              "dw_bwd: add_half size");
  TORCH_CHECK(!mask_x || relu, "dw_bwd: mask_x needs the ReLU'd input");
  TORCH_CHECK(dx.numel() == dy.numel() && w.numel() == 9 * C, "dw_bwd sizes");
  ok(dw_bwd(p, stream()), "dw_bwd");
}

// calls: a list of dw_wgrad argument tuples (x, dy, dw, ab, relu, B, H, W, C, replicas, algo) -> one grouped launch
void dw_wgrad_batch_op(py::list calls) {
  std::vector<DwParams> ps;
  for (auto h : calls) {
    auto t = h.cast<py::tuple>();
    TORCH_CHECK(t.size() == 11, "dw_wgrad_batch: each call needs the 11 dw_wgrad arguments");
    OptT ab = t[3].is_none() ? OptT() : OptT(t[3].cast<at::Tensor>());
    ps.push_back(dw_wgrad_params(t[0].cast<at::Tensor>(), t[1].cast<at::Tensor>(), t[2].cast<at::Tensor>(), ab,
                                 t[4].cast<int>(), t[5].cast<int>(), t[6].cast<int>(), t[7].cast<int>(),
                                 t[8].cast<int>(), t[9].cast<int>(), t[10].cast<int>()));
  }
  ok(dw_wgrad_batch(ps.data(), (int)ps.size(), stream()), "dw_wgrad_batch");
}

void entry_fwd_op(at::Tensor images, at::Tensor idx, at::Tensor w, at::Tensor bias, at::Tensor y, OptT stats, int B,
                  int S, int Cout) {
  EntryParams p{};
  p.images = ptr<const uint8_t>(images, "images");
  p.idx = ptr<const int32_t>(idx, "idx");
  p.w = ptr<const float>(w, "w");
  p.bias = ptr<const float>(bias, "bias");
  p.y = ptr<bf16_t>(y, "y");
  p.stats = optr<float>(stats, "stats");
  p.B = B; p.S = S; p.Cout = Cout; p.Ho = (S + 1) / 2; p.Wo = (S + 1) / 2;
  TORCH_CHECK(idx.numel() == B && y.numel() == (int64_t)B * p.Ho * p.Wo * Cout && w.numel() == 27 * Cout, "entry_fwd sizes");
  ok(entry_fwd(p, stream()), "entry_fwd");
}

// bwd_y given: dy is the gradient w.r.t. the entry BN's output and the operand its BN-backward apply (folded into
// the dy load; bwd_dx is only written by the unfolded fallback)
void entry_wgrad_op(at::Tensor images, at::Tensor idx, at::Tensor dy, at::Tensor dw, int B, int S, int Cout,
                    int replicas, OptT bwd_y, OptT bwd_ab, OptT bwd_sums, int bwd_reps, OptT bwd_dx, OptT bwd_dgamma,
                    OptT bwd_dbeta) {
  EntryParams p{};
  p.replicas = replicas < 1 ? 1 : replicas;
  p.images = ptr<const uint8_t>(images, "images");
  p.idx = ptr<const int32_t>(idx, "idx");
  p.dy = ptr<const bf16_t>(dy, "dy");
  p.dw = ptr<float>(dw, "dw");
  p.B = B; p.S = S; p.Cout = Cout; p.Ho = (S + 1) / 2; p.Wo = (S + 1) / 2;
  TORCH_CHECK(dy.numel() == (int64_t)B * p.Ho * p.Wo * Cout &&
                  dw.numel() == (cfl_det_host() ? 2 : 1) * (int64_t)p.replicas * 27 * Cout,
              "entry_wgrad sizes");
  if (bwd_y) {
    TORCH_CHECK(bwd_ab && bwd_sums, "entry_wgrad: bwd_y needs bwd_ab and bwd_sums");
    TORCH_CHECK(Cout <= BNB_MAX_C && bwd_reps >= 1 && bwd_reps <= BNB_MAX_REPS && bwd_y->numel() == dy.numel() &&
                bwd_ab->numel() >= 4 * Cout && bwd_sums->numel() >= (int64_t)bwd_reps * 2 * Cout &&
                (!bwd_dx || bwd_dx->numel() == dy.numel()) && (!bwd_dgamma || bwd_dgamma->numel() >= Cout) &&
                (!bwd_dbeta || bwd_dbeta->numel() >= Cout), "entry_wgrad: bwd tensor sizes");
    p.bwd.y = ptr<const bf16_t>(*bwd_y, "bwd_y");
    p.bwd.ab = ptr<const float>(*bwd_ab, "bwd_ab");
    p.bwd.sums = ptr<const float>(*bwd_sums, "bwd_sums");
    p.bwd.reps = bwd_reps;
    p.bwd.invM = 1.f / (float)((int64_t)B * p.Ho * p.Wo);
    p.bwd.dx = optr<bf16_t>(bwd_dx, "bwd_dx");
    p.bwd.dgamma = optr<float>(bwd_dgamma, "bwd_dgamma");
    p.bwd.dbeta = optr<float>(bwd_dbeta, "bwd_dbeta");
  }
  ok(entry_wgrad(p, stream()), "entry_wgrad");
}

void bn_finalize_op(OptT stats, at::Tensor gamma, at::Tensor beta, at::Tensor mm, at::Tensor mv, at::Tensor ab, int C,
                    double count, double eps, int train) {
  TORCH_CHECK(ab.numel() >= 4 * C, "bn_finalize: ab size");
  ok(bn_finalize(optr<const float>(stats, "stats"), ptr<const float>(gamma, "gamma"), ptr<const float>(beta, "beta"),
                 ptr<const float>(mm, "mm"), ptr<const float>(mv, "mv"), ptr<float>(ab, "ab"), C, (float)count,
                 (float)eps, train, stream()),
     "bn_finalize");
}

// layers: list of (stats, moving_mean, moving_var, C, count) -> device table (uint8 tensor)
at::Tensor make_bn_moving_table(std::vector<std::tuple<at::Tensor, at::Tensor, at::Tensor, int, double>> layers) {
  std::vector<BnMoving> h;
  at::Device dev = std::get<0>(layers.at(0)).device();
  for (auto& l : layers) {
    BnMoving b{};
    b.stats = ptr<const float>(std::get<0>(l), "stats");
    b.mmean = ptr<float>(std::get<1>(l), "mmean");
    b.mvar = ptr<float>(std::get<2>(l), "mvar");
    b.C = std::get<3>(l);
    TORCH_CHECK(b.C > 0 && b.C <= 1024 && 1024 % b.C == 0, "bn moving table: C must divide 1024");
    b.count = (float)std::get<4>(l);
    h.push_back(b);
  }
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(BnMoving))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(BnMoving));
  return cpu.to(dev);
}

// layers: list of (gamma, beta, moving_mean, moving_var, ab, C) -> device table (uint8 tensor)
at::Tensor make_bn_eval_table(std::vector<std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, int>> layers,
                              double eps) {
  std::vector<BnEval> h;
  at::Device dev = std::get<0>(layers.at(0)).device();
  for (auto& l : layers) {
    BnEval b{};
    b.gamma = ptr<const float>(std::get<0>(l), "gamma");
    b.beta = ptr<const float>(std::get<1>(l), "beta");
    b.mmean = ptr<const float>(std::get<2>(l), "mmean");
    b.mvar = ptr<const float>(std::get<3>(l), "mvar");
    b.ab = ptr<float>(std::get<4>(l), "ab");
    b.C = std::get<5>(l);
    TORCH_CHECK(std::get<4>(l).numel() >= 4 * b.C && std::get<0>(l).numel() == b.C, "bn eval table: sizes");
    b.eps = (float)eps;
    h.push_back(b);
  }
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(BnEval))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(BnEval));
  return cpu.to(dev);
}

void bn_eval_coefs_op(at::Tensor table, int n_layers) {
  TORCH_CHECK(table.numel() == (int64_t)n_layers * (int64_t)sizeof(BnEval), "bn_eval_coefs: table size");
  ok(bn_eval_coefs(ptr<const BnEval>(table, "table"), n_layers, stream()), "bn_eval_coefs");
}

void bn_moving_update_op(at::Tensor table, int n_layers, double momentum) {
  TORCH_CHECK(table.numel() == (int64_t)n_layers * (int64_t)sizeof(BnMoving), "bn_moving_update: table size");
  ok(bn_moving_update(ptr<const BnMoving>(table, "table"), n_layers, 0, (float)momentum, stream()), "bn_moving_update");
}

void node_bwd_op(OptT src0, int mode0, int mask0, OptT src1, int mode1, int mask1, OptT argmax, at::Tensor v, OptT ab,
                 int relu_node, at::Tensor out, OptT sums, int B, int H, int W, int C, int sum_reps, OptT sy,
                 OptT sab) {
  NodeBwdParams p{};
  p.sy = optr<const bf16_t>(sy, "sy");
  p.sab = optr<const float>(sab, "sab");
  TORCH_CHECK(!p.sy || (p.sab && sy->numel() == out.numel() && sab->numel() >= 4 * C), "node_bwd: sy / sab");
  p.sum_reps = sum_reps < 1 ? 1 : sum_reps;
  p.src[0] = GradSrc{optr<const bf16_t>(src0, "src0"), src0.has_value() ? mode0 : 0, mask0};
  p.src[1] = GradSrc{optr<const bf16_t>(src1, "src1"), src1.has_value() ? mode1 : 0, mask1};
  if (!p.src[0].p) p.src[0].mode = GM_NONE;
  if (!p.src[1].p) p.src[1].mode = GM_NONE;
  p.argmax = optr<const uint8_t>(argmax, "argmax");
  p.v = ptr<const bf16_t>(v, "v");
  p.ab = optr<const float>(ab, "ab");
  p.relu_node = relu_node;
  p.out = ptr<bf16_t>(out, "out");
  p.sums = optr<float>(sums, "sums");
  p.B = B; p.H = H; p.W = W; p.C = C;
  const int64_t n = (int64_t)B * H * W * C;
  TORCH_CHECK(v.numel() == n && out.numel() == n, "node_bwd: v/out size");
  if (sums) TORCH_CHECK(sums->numel() >= (int64_t)p.sum_reps * (ab || sab ? 2 : 1) * C, "node_bwd: sums size");
  const int64_t half = (int64_t)B * ((H + 1) / 2) * ((W + 1) / 2) * C;
  for (int s = 0; s < 2; ++s) {
    const OptT& t = s ? src1 : src0;
    if (!p.src[s].p) continue;
    const int m = p.src[s].mode;
    const int64_t want = m == GM_SAME ? n : m == GM_SUM2X2 ? 4 * n : half;
    TORCH_CHECK(t->numel() == want, "node_bwd: source ", s, " size ", t->numel(), " != ", want);
    if (m == GM_MAXPOOL) TORCH_CHECK(p.argmax && argmax->numel() == half, "node_bwd: argmax size");
  }
  ok(node_bwd(p, stream()), "node_bwd");
}

void bn_bwd_apply_op(at::Tensor g, at::Tensor y, at::Tensor ab, at::Tensor sums, at::Tensor dy, OptT dgamma,
                     OptT dbeta, int M, int C, int sum_reps) {
  ok(bn_bwd_apply(bba_params(g, y, ab, sums, dy, dgamma, dbeta, M, C, sum_reps), stream()), "bn_bwd_apply");
}

void pool_res_fwd_op(at::Tensor y, at::Tensor ab, at::Tensor res, at::Tensor out, at::Tensor argmax, int B, int H,
                     int W, int C) {
  PoolResParams p{};
  p.y = ptr<const bf16_t>(y, "y");
  p.ab = ptr<const float>(ab, "ab");
  p.res = ptr<const bf16_t>(res, "res");
  p.out = ptr<bf16_t>(out, "out");
  p.argmax = ptr<uint8_t>(argmax, "argmax");
  p.B = B; p.H = H; p.W = W; p.C = C; p.Ho = (H + 1) / 2; p.Wo = (W + 1) / 2;
  const int64_t no = (int64_t)B * p.Ho * p.Wo * C;
  TORCH_CHECK(y.numel() == (int64_t)B * H * W * C && res.numel() == no && out.numel() == no && argmax.numel() == no,
              "pool_res_fwd sizes");
  ok(pool_res_fwd(p, stream()), "pool_res_fwd");
}

void bn_add_fwd_op(at::Tensor y, at::Tensor ab, at::Tensor q, int q_up, at::Tensor out, int B, int H, int W, int C) {
  BnAddParams p{};
  p.y = ptr<const bf16_t>(y, "y");
  p.ab = ptr<const float>(ab, "ab");
  p.q = ptr<const bf16_t>(q, "q");
  p.q_up = q_up;
  p.out = ptr<bf16_t>(out, "out");
  p.B = B; p.H = H; p.W = W; p.C = C;
  const int64_t n = (int64_t)B * H * W * C;
  TORCH_CHECK(y.numel() == n && out.numel() == n && q.numel() == (q_up ? n / 4 : n), "bn_add_fwd sizes");
  ok(bn_add_fwd(p, stream()), "bn_add_fwd");
}

HeadParams headp(at::Tensor x, at::Tensor w, at::Tensor bias, at::Tensor masks, at::Tensor idx, at::Tensor h,
                 at::Tensor metrics, int B, int R, int Cin, int dice) {
  HeadParams p{};
  p.x = ptr<const bf16_t>(x, "x");
  p.w = ptr<const float>(w, "w");
  p.bias = ptr<const float>(bias, "bias");
  p.masks = ptr<const uint8_t>(masks, "masks");
  p.idx = ptr<const int32_t>(idx, "idx");
  p.h = ptr<float>(h, "h");
  p.metrics = ptr<double>(metrics, "metrics");
  p.B = B; p.R = R; p.Cin = Cin; p.dice = dice;
  TORCH_CHECK(x.numel() == (int64_t)B * R * R * Cin && h.numel() == (int64_t)B * R * R && idx.numel() == B &&
              metrics.numel() >= 10 && masks.size(-1) == 2 * R, "head sizes");
  return p;
}

void head_fwd_op(at::Tensor x, at::Tensor w, at::Tensor bias, at::Tensor masks, at::Tensor idx, at::Tensor h,
                 at::Tensor metrics, int B, int R, int Cin, int dice) {
  ok(head_fwd(headp(x, w, bias, masks, idx, h, metrics, B, R, Cin, dice), stream()), "head_fwd");
}

void head_bwd_op(at::Tensor x, at::Tensor w, at::Tensor bias, at::Tensor masks, at::Tensor idx, at::Tensor h,
                 at::Tensor metrics, at::Tensor dx, at::Tensor dw, at::Tensor db, int B, int R, int Cin, int dice,
                 OptT node_y, OptT node_ab, OptT node_sums, int node_reps, int fused, OptT dwfx) {
  HeadParams p = headp(x, w, bias, masks, idx, h, metrics, B, R, Cin, dice);
  p.fused = fused;
  p.dx = ptr<bf16_t>(dx, "dx");
  p.dw = ptr<float>(dw, "dw");
  p.db = ptr<float>(db, "db");
  if (cfl_det_host()) {               // deterministic mode: dW / db accumulate as int64 fixed point (GF_FIXED)
    TORCH_CHECK(dwfx.has_value() && dwfx->numel() >= 2 * (Cin + 1), "head_bwd: the deterministic mode needs dwfx");
    p.dwfx = ptr<float>(*dwfx, "dwfx");
  }
  TORCH_CHECK(dx.numel() == x.numel(), "head_bwd: dx size");
  p.node = node_epi_args(node_y, node_ab, node_sums, node_reps, 0, dx.numel(), Cin);
  ok(head_bwd(p, stream()), "head_bwd");
}

void adam_update_op(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor trainable, double lr, double b1,
                    double b2, double eps, at::Tensor step) {
  AdamParams a{};
  a.p = ptr<float>(p, "p");
  a.g = ptr<const float>(g, "g");
  a.m = ptr<float>(m, "m");
  a.v = ptr<float>(v, "v");
  a.trainable = ptr<const uint8_t>(trainable, "trainable");
  a.n = p.numel();
  a.lr = (float)lr; a.b1 = (float)b1; a.b2 = (float)b2; a.eps = (float)eps;
  a.step = ptr<int>(step, "step");
  TORCH_CHECK(g.numel() == a.n && m.numel() == a.n && v.numel() == a.n && trainable.numel() == a.n, "adam sizes");
  ok(adam_update(a, stream()), "adam_update");
}

void adam_step_done_op(at::Tensor step) { ok(adam_step_done(ptr<int>(step, "step"), stream()), "adam_step_done"); }

// views: list of (kind, src_offset, dst_offset, ks, cin, cout)
at::Tensor make_pack_table(std::vector<std::tuple<int, int64_t, int64_t, int, int, int>> views, at::Tensor like) {
  std::vector<PackView> h;
  for (auto& v : views) {
    PackView p{};
    p.kind = std::get<0>(v); p.src = std::get<1>(v); p.dst = std::get<2>(v);
    p.ks = std::get<3>(v); p.cin = std::get<4>(v); p.cout = std::get<5>(v);
    h.push_back(p);
  }
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(PackView))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(PackView));
  return cpu.to(like.device());
}

void pack_weights_op(at::Tensor flat, at::Tensor packed, at::Tensor table, int n_views, int max_elems, OptT step,
                     OptT cursor) {
  TORCH_CHECK(table.numel() == (int64_t)n_views * (int64_t)sizeof(PackView), "pack: table size");
  ok(pack_weights(ptr<const float>(flat, "flat"), ptr<bf16_t>(packed, "packed"), ptr<const PackView>(table, "table"),
                  n_views, max_elems, stream(), optr<int>(step, "step"), optr<int>(cursor, "cursor")),
     "pack_weights");
}

// items: list of (kind, n, r0, c0, rows, cols, q, s1, s2, base2, src, dst_t, dst_b) for OI_FLAT / OI_TILE, then one
// OI_MOVING item per (stats, moving_mean, moving_variance, C, count)
at::Tensor make_opt_table(std::vector<std::tuple<int, int, int, int, int, int, int, int, int, int, int64_t, int64_t,
                                                 int64_t>> items,
                          std::vector<std::tuple<at::Tensor, at::Tensor, at::Tensor, int, double>> moving,
                          at::Tensor like) {
  std::vector<OptItem> h;
  for (auto& t : items) {
    OptItem o{};
    o.kind = std::get<0>(t); o.n = std::get<1>(t); o.r0 = std::get<2>(t); o.c0 = std::get<3>(t);
    o.rows = std::get<4>(t); o.cols = std::get<5>(t); o.q = std::get<6>(t); o.s1 = std::get<7>(t);
    o.s2 = std::get<8>(t); o.base2 = std::get<9>(t); o.src = std::get<10>(t); o.dst_t = std::get<11>(t);
    o.dst_b = std::get<12>(t);
    TORCH_CHECK(o.kind == OI_FLAT || o.kind == OI_TILE, "opt table: kind");
    TORCH_CHECK(o.kind != OI_FLAT || (o.n > 0 && o.n <= 1024), "opt table: flat items hold 1..1024 elements");
    TORCH_CHECK(o.kind != OI_TILE || (o.q > 0 && o.rows > 0 && o.cols > 0 && o.r0 % 64 == 0 && o.c0 % 64 == 0 &&
                                      o.r0 < o.rows && o.c0 < o.cols), "opt table: tile geometry");
    h.push_back(o);
  }
  for (auto& l : moving) {
    OptItem o{};
    o.kind = OI_MOVING;
    o.stats = ptr<const float>(std::get<0>(l), "stats");
    o.mmean = ptr<float>(std::get<1>(l), "mmean");
    o.mvar = ptr<float>(std::get<2>(l), "mvar");
    o.n = std::get<3>(l);
    o.count = (float)std::get<4>(l);
    TORCH_CHECK(std::get<0>(l).numel() >= (int64_t)STAT_REPLICAS * 2 * o.n && std::get<1>(l).numel() >= o.n &&
                std::get<2>(l).numel() >= o.n, "opt table: moving sizes");
    h.push_back(o);
  }
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(OptItem))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(OptItem));
  return cpu.to(like.device());
}

void opt_step_op(at::Tensor table, int n_items, at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v,
                 at::Tensor trainable, at::Tensor packed, double lr, double b1, double b2, double eps, double momentum,
                 OptT step, OptT cursor, OptT ticket, OptT lr_buf) {
  TORCH_CHECK(table.numel() == (int64_t)n_items * (int64_t)sizeof(OptItem), "opt_step: table size");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel() &&
              trainable.numel() == p.numel(), "opt_step sizes");
  OptParams o{};
  o.p = ptr<float>(p, "p");
  o.g = ptr<const float>(g, "g");
  o.m = ptr<float>(m, "m");
  o.v = ptr<float>(v, "v");
  o.trainable = ptr<const uint8_t>(trainable, "trainable");
  o.packed = ptr<bf16_t>(packed, "packed");
  o.items = ptr<const OptItem>(table, "table");
  o.n_items = n_items;
  o.lr = (float)lr; o.b1 = (float)b1; o.b2 = (float)b2; o.eps = (float)eps; o.momentum = (float)momentum;
  o.step = optr<int>(step, "step");
  o.cursor = optr<int>(cursor, "cursor");
  o.ticket = optr<int>(ticket, "ticket");
  o.lr_t = optr<const float>(lr_buf, "lr_buf");
  TORCH_CHECK(lr_buf ? !step && !cursor : step && ticket,
              "opt_step: either step + ticket (+ cursor), or lr_buf alone (zero_spans advanced the step)");
  ok(opt_step(o, stream()), "opt_step");
}

// entries: list of (src, dst, n, replicas, mode) -> (device table, grid size)
std::tuple<at::Tensor, int> make_grad_finish_table(std::vector<std::tuple<at::Tensor, at::Tensor, int, int, int>> entries) {
  std::vector<GradFinish> h;
  at::Device dev = std::get<0>(entries.at(0)).device();
  for (auto& e : entries) {
    GradFinish g{};
    g.src = ptr<float>(std::get<0>(e), "src");
    g.dst = ptr<float>(std::get<1>(e), "dst");
    g.n = std::get<2>(e); g.replicas = std::get<3>(e); g.mode = std::get<4>(e);
    TORCH_CHECK(g.mode >= GF_REDUCE && g.mode <= GF_FIXED, "grad_finish: mode");
    TORCH_CHECK(g.mode != GF_FIXED || cfl_det_host(), "grad_finish: GF_FIXED entries need the deterministic mode");
    TORCH_CHECK(g.mode == GF_FIXED || (g.n % 4 == 0 && (reinterpret_cast<uintptr_t>(g.src) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(g.dst) & 15) == 0), "grad_finish: n % 4 and 16-byte alignment");
    TORCH_CHECK(std::get<1>(e).numel() >= g.n, "grad_finish: dst size");
    // deterministic mode: REDUCE / FIXED sources are int64 fixed-point elements (two floats each)
    const int64_t w = cfl_det_host() && (g.mode == GF_REDUCE || g.mode == GF_FIXED) ? 2 : 1;
    TORCH_CHECK(std::get<0>(e).numel() >= w * g.n * (g.mode == GF_COPY || g.mode == GF_FIXED ? 1 : g.replicas),
                "grad_finish: src size");
    h.push_back(g);
  }
  TORCH_CHECK(h.size() <= 256, "grad_finish: at most 256 entries");
  const int work = grad_finish_work(h.data(), (int)h.size());
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(GradFinish))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(GradFinish));
  return {cpu.to(dev), work};
}

void grad_finish_op(at::Tensor table, int n_entries, int total_work) {
  TORCH_CHECK(table.numel() == (int64_t)n_entries * (int64_t)sizeof(GradFinish), "grad_finish: table size");
  ok(grad_finish(ptr<const GradFinish>(table, "table"), n_entries, total_work, stream()), "grad_finish");
}

at::Tensor make_zero_table(std::vector<at::Tensor> spans) {
  std::vector<ZeroSpan> h;
  for (auto& t : spans) {
    ZeroSpan z{};
    z.p = t.data_ptr();
    z.bytes = t.numel() * t.element_size();
    TORCH_CHECK(t.is_contiguous() && (reinterpret_cast<uintptr_t>(z.p) & 15) == 0 && z.bytes % 16 == 0,
                "zero_spans: spans must be contiguous, 16-byte aligned, multiple of 16 bytes");
    h.push_back(z);
  }
  auto cpu = torch::empty({(int64_t)(h.size() * sizeof(ZeroSpan))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), h.data(), h.size() * sizeof(ZeroSpan));
  return cpu.to(spans.at(0).device());
}

void zero_spans_op(at::Tensor table, int n, int64_t max_bytes, OptT batches, OptT cursor, OptT idx, OptT step,
                   OptT lr_buf, double lr, double b1, double b2) {
  TORCH_CHECK(table.numel() == (int64_t)n * (int64_t)sizeof(ZeroSpan), "zero_spans: table size");
  BatchSelect bs{};
  if (batches) {
    TORCH_CHECK(cursor && idx && batches->dim() == 2 && batches->size(1) == idx->numel() &&
                batches->scalar_type() == at::kInt && idx->scalar_type() == at::kInt && cursor->numel() >= 1,
                "zero_spans: batches [nb][B] int32 with cursor and idx [B]");
    bs.table = ptr<const int32_t>(*batches, "batches");
    bs.cursor = ptr<int>(*cursor, "cursor");
    bs.idx = ptr<int32_t>(*idx, "idx");
    bs.B = (int)idx->numel();
    bs.nb = (int)batches->size(0);
  }
  StepAdvance adv{};
  if (step) {
    TORCH_CHECK(lr_buf && lr_buf->numel() >= 1 && lr_buf->scalar_type() == at::kFloat && step->numel() >= 1 &&
                step->scalar_type() == at::kInt, "zero_spans: step advance needs int32 step and float32 lr_buf");
    adv.step = ptr<int>(*step, "step");
    adv.lr_t = ptr<float>(*lr_buf, "lr_buf");
    adv.lr = (float)lr; adv.b1 = (float)b1; adv.b2 = (float)b2;
  }
  ok(zero_spans(ptr<const ZeroSpan>(table, "table"), n, max_bytes, stream(), bs, adv), "zero_spans");
}

// src: uint8 device bytes of n decoded images back to back; offs: int64 [n] byte offsets; dims: int32 [n, 2] (h, w);
// dst: uint8 [n, dh, dw, c] or [n, dh, dw] (c = 1)
void resize_batch_op(at::Tensor src, at::Tensor offs, at::Tensor dims, at::Tensor dst, int binarize) {
  TORCH_CHECK(src.scalar_type() == at::kByte && dst.scalar_type() == at::kByte, "resize_batch: uint8 tensors");
  TORCH_CHECK(offs.scalar_type() == at::kLong && dims.scalar_type() == at::kInt, "resize_batch: offs int64, dims int32");
  const int n = (int)offs.numel();
  TORCH_CHECK(dims.numel() == 2 * n && dst.dim() >= 3 && dst.size(0) == n, "resize_batch: shapes");
  const int dh = (int)dst.size(1), dw = (int)dst.size(2), c = dst.dim() == 4 ? (int)dst.size(3) : 1;
  ok(resize_batch(ptr<const uint8_t>(src, "src"), ptr<const int64_t>(offs, "offs"), ptr<const int>(dims, "dims"),
                  ptr<uint8_t>(dst, "dst"), n, dh, dw, c, binarize, stream()), "resize_batch");
}

void render_cracks_op(at::Tensor segs, at::Tensor params, at::Tensor images, at::Tensor masks, int n, int img,
                      int max_seg) {
  TORCH_CHECK(images.numel() == (int64_t)n * img * img * 3 && masks.numel() == (int64_t)n * img * img &&
              segs.numel() == (int64_t)n * max_seg * 6 && params.numel() == (int64_t)n * 8, "render sizes");
  ok(render_cracks(ptr<const float>(segs, "segs"), ptr<const float>(params, "params"), ptr<uint8_t>(images, "images"),
                   ptr<uint8_t>(masks, "masks"), n, img, max_seg, stream()),
     "render_cracks");
}

void gather_rows_u8_op(at::Tensor src, at::Tensor idx, at::Tensor dst, int64_t row_bytes) {
  TORCH_CHECK(dst.numel() == idx.numel() * row_bytes, "gather_rows sizes");
  ok(gather_rows_u8(ptr<const uint8_t>(src, "src"), ptr<const int32_t>(idx, "idx"), ptr<uint8_t>(dst, "dst"),
                    (int)idx.numel(), row_bytes, stream()),
     "gather_rows_u8");
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "CDNA4 (gfx950) HIP kernels of the crack-segmentation FL trainer";
  m.attr("STAT_REPLICAS") = STAT_REPLICAS;
  m.def("conv_igemm", &conv_igemm_op, py::arg("x"), py::arg("wt"), py::arg("bias"), py::arg("y"), py::arg("stats"),
        py::arg("ab"), py::arg("relu"), py::arg("B"), py::arg("Hin"), py::arg("Win"), py::arg("Cin"), py::arg("up_in"),
        py::arg("Ho"), py::arg("Wo"), py::arg("N"), py::arg("ks"), py::arg("stride"), py::arg("pad_t"),
        py::arg("pad_l"), py::arg("ws") = py::none(), py::arg("algo") = 0, py::arg("node_y") = py::none(),
        py::arg("node_ab") = py::none(), py::arg("node_sums") = py::none(), py::arg("node_reps") = 1,
        py::arg("node_relu") = 1, py::arg("join_mode") = 0, py::arg("join_y") = py::none(),
        py::arg("join_ab") = py::none(), py::arg("join_out") = py::none(), py::arg("join_argmax") = py::none(),
        py::arg("join_H") = 0, py::arg("join_W") = 0,
        py::arg("bwd_y") = py::none(), py::arg("bwd_ab") = py::none(), py::arg("bwd_sums") = py::none(),
        py::arg("bwd_reps") = 1, py::arg("bwd_dx") = py::none(), py::arg("bwd_dgamma") = py::none(),
        py::arg("bwd_dbeta") = py::none(), py::arg("pj_v") = py::none(), py::arg("pj_add") = py::none(),
        py::arg("pj_out") = py::none(), py::arg("pj_sy") = py::none(), py::arg("pj_sab") = py::none(),
        py::arg("pj_sums") = py::none(), py::arg("pj_reps") = 1, py::arg("jfin_stats") = py::none(),
        py::arg("jfin_gamma") = py::none(), py::arg("jfin_beta") = py::none(), py::arg("jfin_count") = 0.0,
        py::arg("jfin_eps") = 1e-3, py::arg("xfin_stats") = py::none(), py::arg("xfin_gamma") = py::none(),
        py::arg("xfin_beta") = py::none(), py::arg("xfin_count") = 0.0, py::arg("xfin_eps") = 1e-3,
        py::arg("sum2x2") = py::none(), py::arg("side_bba") = py::none(), py::arg("side_pool") = py::none(),
        py::arg("wt8") = py::none(), py::arg("ws8") = py::none());
  m.def("quant_w8", [](py::list views) {
    // [(src bf16 [N][K] as int16, dst uint8 [N][K], scales uint8 [N][K/32]), ...] in ONE launch
    std::vector<const bf16_t*> src;
    std::vector<uint8_t*> dst, sc;
    std::vector<int> nblk;
    for (auto h : views) {
      const py::tuple t = h.cast<py::tuple>();
      TORCH_CHECK(t.size() == 3, "quant_w8: (src, dst, scales)");
      const at::Tensor a = t[0].cast<at::Tensor>(), d = t[1].cast<at::Tensor>(), c = t[2].cast<at::Tensor>();
      TORCH_CHECK(a.numel() % 32 == 0 && d.numel() >= a.numel() && c.numel() >= a.numel() / 32 &&
                  d.scalar_type() == at::kByte && c.scalar_type() == at::kByte, "quant_w8: sizes / dtypes");
      src.push_back(ptr<const bf16_t>(a, "src"));
      dst.push_back(ptr<uint8_t>(d, "dst"));
      sc.push_back(ptr<uint8_t>(c, "scales"));
      nblk.push_back((int)(a.numel() / 32));
    }
    ok(quant_w8(src.data(), dst.data(), sc.data(), nblk.data(), (int)src.size(), stream()), "quant_w8");
  }, "e4m3 + e8m0-per-32 quantisation of packed bf16 weight views (fp8.hip), one launch");
  m.attr("JOIN_POOL") = (int)JOIN_POOL;
  m.attr("JOIN_ADD") = (int)JOIN_ADD;
  m.attr("JOIN_ADD_UP") = (int)JOIN_ADD_UP;
  m.def("conv_splits", &conv_splits_op);
  m.def("conv_wgrad", &conv_wgrad_op, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("ab"), py::arg("relu"),
        py::arg("B"), py::arg("Hin"), py::arg("Win"), py::arg("Cin"), py::arg("up_in"), py::arg("Ho"), py::arg("Wo"),
        py::arg("N"), py::arg("ks"), py::arg("stride"), py::arg("pad_t"), py::arg("pad_l"), py::arg("dst_mode"),
        py::arg("m_chunk") = 0, py::arg("algo") = 0, py::arg("slabs") = 0);
  m.def("conv_wgrad_batch", &conv_wgrad_batch_op, py::arg("calls"));
  m.def("pw_bwd_supported", &pw_bwd_supported_op);
  m.def("pw_bwd", &pw_bwd_op, py::arg("g"), py::arg("y"), py::arg("ab"), py::arg("sums"), py::arg("reps"),
        py::arg("w"), py::arg("d"), py::arg("dd"), py::arg("dw"), py::arg("replicas"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("K"), py::arg("N"));
  m.def("conv_wgrad_slabs", &conv_wgrad_slabs_op, py::arg("B"), py::arg("Hin"), py::arg("Win"), py::arg("Cin"),
        py::arg("up_in"), py::arg("Ho"), py::arg("Wo"), py::arg("N"), py::arg("ks"), py::arg("stride"),
        py::arg("pad_t"), py::arg("pad_l"), py::arg("algo") = 0);
  m.attr("GF_SUM") = (int)GF_SUM;
  m.attr("TUNE_WGRAD3_BLOCKS") = (int)TUNE_WGRAD3_BLOCKS;
  m.attr("TUNE_WGRAD3_MINTILES") = (int)TUNE_WGRAD3_MINTILES;
  m.def("sep_fwd_supported", &sep_fwd_supported_op, py::arg("B"), py::arg("H"), py::arg("W"), py::arg("K"),
        py::arg("N"));
  m.def("sep_fwd", &sep_fwd_op, py::arg("x"), py::arg("ab"), py::arg("relu"), py::arg("wdw"), py::arg("wpw"),
        py::arg("bias"), py::arg("d"), py::arg("y"), py::arg("stats"), py::arg("B"), py::arg("H"), py::arg("W"),
        py::arg("K"), py::arg("N"), py::arg("xfin_stats") = py::none(), py::arg("xfin_gamma") = py::none(),
        py::arg("xfin_beta") = py::none(), py::arg("xfin_count") = 0.0, py::arg("xfin_eps") = 1e-3);
  m.attr("TUNE_SEP") = (int)TUNE_SEP;
  m.attr("TUNE_SEP_BLOCKS") = (int)TUNE_SEP_BLOCKS;
  m.def("dw_fwd", &dw_fwd_op, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("ab"), py::arg("relu"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("C"), py::arg("algo") = 0, py::arg("xfin_stats") = py::none(),
        py::arg("xfin_gamma") = py::none(), py::arg("xfin_beta") = py::none(), py::arg("xfin_count") = 0.0,
        py::arg("xfin_eps") = 1e-3);
  m.def("dw_dgrad", &dw_dgrad_op, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("B"), py::arg("H"),
        py::arg("W"), py::arg("C"), py::arg("algo") = 0, py::arg("node_y") = py::none(),
        py::arg("node_ab") = py::none(), py::arg("node_sums") = py::none(), py::arg("node_reps") = 1,
        py::arg("node_relu") = 1);
  m.def("dw_wgrad", &dw_wgrad_op, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("ab"), py::arg("relu"),
        py::arg("B"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("replicas") = 1, py::arg("algo") = 0);
  m.def("dw_wgrad_batch", &dw_wgrad_batch_op, py::arg("calls"));
  m.def("dw_bwd", &dw_bwd_op, py::arg("x"), py::arg("ab"), py::arg("relu"), py::arg("dy"), py::arg("w"),
        py::arg("dx"), py::arg("dw"), py::arg("replicas"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("C"),
        py::arg("algo") = 0, py::arg("node_y") = py::none(), py::arg("node_ab") = py::none(),
        py::arg("node_sums") = py::none(), py::arg("node_reps") = 1, py::arg("node_relu") = 1,
        py::arg("add_half") = py::none(), py::arg("mask_x") = 0);
  m.def("entry_fwd", &entry_fwd_op, py::arg("images"), py::arg("idx"), py::arg("w"), py::arg("bias"), py::arg("y"),
        py::arg("stats"), py::arg("B"), py::arg("S"), py::arg("Cout"));
  m.def("entry_wgrad", &entry_wgrad_op, py::arg("images"), py::arg("idx"), py::arg("dy"), py::arg("dw"), py::arg("B"),
        py::arg("S"), py::arg("Cout"), py::arg("replicas") = 1, py::arg("bwd_y") = py::none(),
        py::arg("bwd_ab") = py::none(), py::arg("bwd_sums") = py::none(), py::arg("bwd_reps") = 1,
        py::arg("bwd_dx") = py::none(), py::arg("bwd_dgamma") = py::none(), py::arg("bwd_dbeta") = py::none());
  m.def("make_grad_finish_table", &make_grad_finish_table);
  m.def("mfma_scale_probe", [](at::Tensor a, at::Tensor b, at::Tensor sa, at::Tensor sb, int shape) {
    TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kInt && a.numel() == 512 && b.numel() == 512 &&
                sa.numel() == 64 && sb.numel() == 64 && b.scalar_type() == at::kInt, "mfma_scale_probe operands");
    auto d = at::zeros({64, shape == 16 ? 4 : 16}, a.options().dtype(at::kFloat));
    ok(mfma_scale_probe(a.data_ptr<int>(), b.data_ptr<int>(), sa.data_ptr<int>(), sb.data_ptr<int>(),
                        d.data_ptr<float>(), shape, stream()), "mfma_scale_probe");
    return d;
  }, "one block-scaled fp8 MFMA (16: 16x16x128, 32: 32x32x64) on raw lane registers");
  m.def("fx_overflow", []() {
    const int r = cfl_fx_overflow();
    ok(r == 3 ? 3 : 0, "fx_overflow");
    return r;
  }, "1 if a deterministic-mode fixed-point add was clamped since the last set_det (common.h red_add)");
  m.def("set_det", [](int v) { ok(cfl_det_set(v), "set_det"); },
        "deterministic reduction mode (int64 fixed-point cross-block sums) on / off; before any graph capture");
  m.def("det", []() { return cfl_det_host(); });
  m.attr("GF_FIXED") = (int)GF_FIXED;
  m.def("grad_finish", &grad_finish_op);
  m.def("make_zero_table", &make_zero_table);
  m.def("zero_spans", &zero_spans_op, py::arg("table"), py::arg("n"), py::arg("max_bytes"),
        py::arg("batches") = py::none(), py::arg("cursor") = py::none(), py::arg("idx") = py::none(),
        py::arg("step") = py::none(), py::arg("lr_buf") = py::none(), py::arg("lr") = 0.0, py::arg("b1") = 0.0,
        py::arg("b2") = 0.0);
  m.def("set_ts", [](py::object buf) {
    if (buf.is_none()) {
      ok(cfl_ts_set(nullptr, 0), "set_ts");
      return;
    }
    torch::Tensor t = buf.cast<torch::Tensor>();
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kInt64 && t.is_contiguous() && t.numel() % 2 == 0,
                "set_ts: contiguous int64 device tensor of [blocks][2]");
    ok(cfl_ts_set(t.data_ptr(), (int)(t.numel() / 2)), "set_ts");
  }, "block timeline buffer ([blocks][2] int64 s_memrealtime stamps per kernel launch) or None = off");
  m.def("set_tune", &cfl_set_tune);
  m.def("get_tune", &cfl_tune);
  m.attr("GF_REDUCE") = (int)GF_REDUCE;
  m.attr("GF_COPY") = (int)GF_COPY;
  m.attr("TUNE_NODE_BWD_BLOCKS") = (int)TUNE_NODE_BWD_BLOCKS;
  m.attr("TUNE_DW_WGRAD_BLOCKS") = (int)TUNE_DW_WGRAD_BLOCKS;
  m.attr("TUNE_ENTRY_WGRAD_BLOCKS") = (int)TUNE_ENTRY_WGRAD_BLOCKS;
  m.attr("TUNE_ENTRY_FWD_BLOCKS") = (int)TUNE_ENTRY_FWD_BLOCKS;
  m.attr("TUNE_DW_STREAM_BLOCKS") = (int)TUNE_DW_STREAM_BLOCKS;
  m.attr("TUNE_CONV3_SMALL") = (int)TUNE_CONV3_SMALL;
  m.attr("TUNE_CONV3_BN") = (int)TUNE_CONV3_BN;
  m.attr("TUNE_NODE_POOL2X2") = (int)TUNE_NODE_POOL2X2;
  m.attr("TUNE_ENTRY_ALGO") = (int)TUNE_ENTRY_ALGO;
  m.attr("TUNE_CONV3_WS") = (int)TUNE_CONV3_WS;
  m.attr("TUNE_CONV3_WS_GRID") = (int)TUNE_CONV3_WS_GRID;
  m.attr("TUNE_WGRAD_GROUP") = (int)TUNE_WGRAD_GROUP;
  m.attr("TUNE_CONV3_DEEP") = (int)TUNE_CONV3_DEEP;
  m.attr("TUNE_CONV3_SK") = (int)TUNE_CONV3_SK;
  m.attr("TUNE_CONV3_SK_CFG") = (int)TUNE_CONV3_SK_CFG;
  m.attr("TUNE_WGRAD_MIX_ONLY") = (int)TUNE_WGRAD_MIX_ONLY;
  m.attr("TUNE_WGRAD_MIX_SKIP") = (int)TUNE_WGRAD_MIX_SKIP;
  m.attr("TUNE_WGRAD_MIX_LIST") = (int)TUNE_WGRAD_MIX_LIST;
  m.attr("TUNE_WGRAD_MIX_ORDER") = (int)TUNE_WGRAD_MIX_ORDER;
  m.attr("TUNE_OPT_SCALAR") = (int)TUNE_OPT_SCALAR;
  m.attr("TUNE_PWB") = (int)TUNE_PWB;
  m.attr("TUNE_PWB_BLOCKS") = (int)TUNE_PWB_BLOCKS;
  m.attr("TUNE_WGRAD_REPS") = (int)TUNE_WGRAD_REPS;
  m.attr("TUNE_CONV3_F8") = (int)TUNE_CONV3_F8;
  m.attr("TUNE_DW_BWD_DMA") = (int)TUNE_DW_BWD_DMA;
  m.attr("TUNE_WGRAD3_WIDE") = (int)TUNE_WGRAD3_WIDE;
  m.attr("TUNE_CONV3_BIG_WAVES") = (int)TUNE_CONV3_BIG_WAVES;
  m.attr("TUNE_WGRAD_DIRECT") = (int)TUNE_WGRAD_DIRECT;
  m.attr("TUNE_HEAD_BLOCKS") = (int)TUNE_HEAD_BLOCKS;
  m.attr("TUNE_IGEMM_CFG") = (int)TUNE_IGEMM_CFG;
  m.attr("TUNE_CONV3_WB") = (int)TUNE_CONV3_WB;
  m.attr("TUNE_WGRAD1_BLOCKS") = (int)TUNE_WGRAD1_BLOCKS;
  m.attr("TUNE_WGRAD1_MINPIX") = (int)TUNE_WGRAD1_MINPIX;
  m.attr("TUNE_NODE_BWD_IPT") = (int)TUNE_NODE_BWD_IPT;
  m.attr("TUNE_DW_BWD_BLOCKS") = (int)TUNE_DW_BWD_BLOCKS;
  m.attr("TUNE_BBA_BLOCKS") = (int)TUNE_BBA_BLOCKS;
  m.attr("TUNE_NODE_POOL_BLOCKS") = (int)TUNE_NODE_POOL_BLOCKS;
  m.attr("TUNE_WGRAD1_RM") = (int)TUNE_WGRAD1_RM;
  m.attr("TUNE_PW") = (int)TUNE_PW;
  m.attr("TUNE_PW_BLOCKS") = (int)TUNE_PW_BLOCKS;
  m.attr("TUNE_PW_DEPTH") = (int)TUNE_PW_DEPTH;
  m.attr("TUNE_NODE_POOL_IPT") = (int)TUNE_NODE_POOL_IPT;
  m.attr("TUNE_WGRAD3_MINTILES32") = (int)TUNE_WGRAD3_MINTILES32;
  m.attr("TUNE_WGRAD_MIX") = (int)TUNE_WGRAD_MIX;
  m.attr("TUNE_WGRAD_MIX_XCD") = (int)TUNE_WGRAD_MIX_XCD;
  m.attr("TUNE_SIDE") = (int)TUNE_SIDE;
  m.attr("TUNE_WGRAD1_BIG") = (int)TUNE_WGRAD1_BIG;
  m.attr("TUNE_CONV3_BIG") = (int)TUNE_CONV3_BIG;
  m.attr("TUNE_PW_NB") = (int)TUNE_PW_NB;
  m.attr("TUNE_CONV3_SPLIT_BLOCKS") = (int)TUNE_CONV3_SPLIT_BLOCKS;
  m.attr("TUNE_CONV3_SPLIT_TARGET") = (int)TUNE_CONV3_SPLIT_TARGET;
  m.def("bn_finalize", &bn_finalize_op);
  m.def("make_bn_moving_table", &make_bn_moving_table);
  m.def("bn_moving_update", &bn_moving_update_op);
  m.def("make_bn_eval_table", &make_bn_eval_table);
  m.def("bn_eval_coefs", &bn_eval_coefs_op);
  m.def("node_bwd", &node_bwd_op, py::arg("src0"), py::arg("mode0"), py::arg("mask0"), py::arg("src1"),
        py::arg("mode1"), py::arg("mask1"), py::arg("argmax"), py::arg("v"), py::arg("ab"), py::arg("relu_node"),
        py::arg("out"), py::arg("sums"), py::arg("B"), py::arg("H"), py::arg("W"), py::arg("C"),
        py::arg("sum_reps") = 1, py::arg("sy") = py::none(), py::arg("sab") = py::none());
  m.def("bn_bwd_apply", &bn_bwd_apply_op, py::arg("g"), py::arg("y"), py::arg("ab"), py::arg("sums"), py::arg("dy"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("M"), py::arg("C"), py::arg("sum_reps") = 1);
  m.attr("SUM_REPLICAS") = 4;    // BN-backward sum replica rows (whole-step A/B: 16 / 8 / 4 / 2 / 1 -> 1.550 / 1.529 / 1.522 / 1.537 / 1.584 ms)
  m.def("pool_res_fwd", &pool_res_fwd_op);
  m.def("bn_add_fwd", &bn_add_fwd_op);
  m.def("head_fwd", &head_fwd_op);
  m.def("head_bwd", &head_bwd_op, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("masks"), py::arg("idx"),
        py::arg("h"), py::arg("metrics"), py::arg("dx"), py::arg("dw"), py::arg("db"), py::arg("B"), py::arg("R"),
        py::arg("Cin"), py::arg("dice"), py::arg("node_y") = py::none(), py::arg("node_ab") = py::none(),
        py::arg("node_sums") = py::none(), py::arg("node_reps") = 1, py::arg("fused") = 0,
        py::arg("dwfx") = py::none());
  m.def("adam_update", &adam_update_op);
  m.def("adam_step_done", &adam_step_done_op);
  m.def("make_pack_table", &make_pack_table);
  m.def("pack_weights", &pack_weights_op, py::arg("flat"), py::arg("packed"), py::arg("table"), py::arg("n_views"),
        py::arg("max_elems"), py::arg("step") = py::none(), py::arg("cursor") = py::none());
  m.def("make_opt_table", &make_opt_table);
  m.def("opt_step", &opt_step_op, py::arg("table"), py::arg("n_items"), py::arg("p"), py::arg("g"), py::arg("m"),
        py::arg("v"), py::arg("trainable"), py::arg("packed"), py::arg("lr"), py::arg("b1"), py::arg("b2"),
        py::arg("eps"), py::arg("momentum"), py::arg("step"), py::arg("cursor"), py::arg("ticket"),
        py::arg("lr_buf") = py::none());
  m.attr("OI_FLAT") = (int)OI_FLAT;
  m.attr("OI_TILE") = (int)OI_TILE;
  m.def("render_cracks", &render_cracks_op);
  m.def("resize_batch", &resize_batch_op, py::arg("src"), py::arg("offs"), py::arg("dims"), py::arg("dst"),
        py::arg("binarize") = 0);
  m.def("gather_rows_u8", &gather_rows_u8_op);
}
