// stale_j_probe.cpp — diagnostic for the round-1 "stale J" report of
// mtg_tube_time_cost through the C++ shim.
//
// Replays the call sequence of tests/cpp TimeCostWithQCQPInnerSolve
// (J(1.05 T) with gradient, J(T0), J(T0) with gradient) on the main.cpp
// geometry many times in one process, with the caller-owned workspace
// provided three ways:
//   plain   hipMalloc per call, hipFree after the device synchronise
//   pool         hipMallocAsync / hipFreeAsync on the null stream around the
//                call, exactly the round-1 Scratch (free enqueued before the
//                shim's hipDeviceSynchronize)
//   pool_sync    the same, but hipFreeAsync only after hipDeviceSynchronize
//   pool_stream  hipMallocAsync / hipFreeAsync and the call on a created
//                (non-null) stream, free enqueued before the synchronise
// Every workspace is poisoned with 0xFF bytes (NaN doubles, int32 -1)
// before the call, so a read of scratch that the call did not write first
// shows up as NaN (or as a status outside MTG_TRAJ_*).  Outputs are
// compared bit for bit with the first plain evaluation.  Output buffers are
// fresh hipMalloc'd per call and pre-filled with a sentinel, as the shim's
// DeviceBuffer would be (the shim does not fill; the sentinel tells "kernel
// never wrote" apart from "stale value").
//
// Build: see tools/stale_j_probe.sh.  Not part of the product or the tests.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mav_tube_trajectory_generation_amd/vertex.h"
#include "mtg_hip.h"

using namespace mav_trajectory_generation;

namespace {

#define HIP_OK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e_));                                     \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

struct Inputs {
  std::vector<double> pos, df, radii, t0;
};

Inputs mainCpp() {
  const double pts[5][3] = {{2.7, 9.5, 4.8},
                            {3.50796, 4.34802, 4.56653},
                            {3.95552, 3.23008, 4.75131},
                            {5.06673, 2.31032, 4.79433},
                            {7.0, 2.2, 4.8}};
  Vertex::Vector vs;
  Inputs in;
  for (int v = 0; v < 5; ++v) {
    Vertex x(3);
    VectorXd p{pts[v][0], pts[v][1], pts[v][2]};
    if (v == 0 || v == 4)
      x.makeStartOrEnd(p, 4);
    else
      x.addConstraint(derivative_order::POSITION, p);
    vs.push_back(x);
    for (int d = 0; d < 3; ++d) in.pos.push_back(pts[v][d]);
  }
  in.t0 = estimateSegmentTimes(vs, 2.0, 2.0);
  in.df.assign(3 * 10, 0.0);
  for (int d = 0; d < 3; ++d) {
    in.df[d * 10 + 0] = pts[0][d];
    in.df[d * 10 + 5] = pts[4][d];
  }
  in.radii.assign(4 * 2, 0.15);
  return in;
}

struct Result {
  double J = 0.0;
  std::vector<double> g;
  int32_t st = -7;
  int overlap = 0;  // live buffers of this call that the workspace overlaps
  bool pts_ok = true;         // evaluation points read back intact (pool_sync)
  double qcost0 = 0, pts0 = 0;
};

template <typename T>
T* upload(const std::vector<T>& v) {
  T* p = nullptr;
  HIP_OK(hipMalloc(&p, v.size() * sizeof(T)));
  HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

Result evaluate(mtg_ctx* ctx, const Inputs& in, const std::vector<double>& t, int grad_mode,
                const std::string& mode) {
  mtg_time_params p{};
  p.time_penalty = 500.0;
  p.increment = 0.1;
  p.w_d = 0.1;
  p.w_t = 1.0;
  p.grad_mode = grad_mode;
  p.soft_weight = 100.0;
  p.soft_maximum_cost = 1e12;
  double *pos = upload(in.pos), *df = upload(in.df), *tcp = upload(in.t0), *tt = upload(t),
         *rad = upload(in.radii);
  const std::vector<double> sentinel(4, 12345.0);
  double* cost = upload(std::vector<double>(1, 12345.0));
  double* grad = upload(sentinel);
  int32_t* st = upload(std::vector<int32_t>(1, -7));
  const int64_t nbytes = mtg_tube_time_workspace_bytes(10, 4, 1, &p, 0);
  if (nbytes < 0) std::exit(3);
  void* ws = nullptr;
  const bool pooled = mode.rfind("pool", 0) == 0;
  hipStream_t s = nullptr;
  if (mode == "pool_stream") HIP_OK(hipStreamCreate(&s));
  if (pooled)
    HIP_OK(hipMallocAsync(&ws, nbytes, s));
  else
    HIP_OK(hipMalloc(&ws, nbytes));
  // Does the workspace overlap any buffer of this call that is still live?
  Result r;
  {
    const char* w0 = static_cast<const char*>(ws);
    const struct {
      const void* p;
      size_t n;
    } live[8] = {{pos, in.pos.size() * 8}, {df, in.df.size() * 8}, {tcp, in.t0.size() * 8},
                 {tt, t.size() * 8},       {rad, in.radii.size() * 8}, {cost, 8},
                 {grad, 32},               {st, 4}};
    for (const auto& b : live) {
      const char* b0 = static_cast<const char*>(b.p);
      if (b0 < w0 + nbytes && w0 < b0 + b.n) ++r.overlap;
    }
  }
  HIP_OK(hipMemsetAsync(ws, 0xFF, nbytes, s));
  const int rc = mtg_tube_time_cost(ctx, 10, 4, 4, 1, pos, df, tcp, tt, rad, 1e-10, 100, &p,
                                    cost, grad_mode ? grad : nullptr, st, ws, nbytes, s);
  if (rc != MTG_OK) {
    std::fprintf(stderr, "mtg_tube_time_cost: %s\n", mtg_status_string(rc));
    std::exit(4);
  }
  if (mode == "pool") HIP_OK(hipFreeAsync(ws, s));
  HIP_OK(hipDeviceSynchronize());
  if (pooled && mode != "pool") {
    // Where did the call go wrong?  Read back the evaluation points and the
    // QCQP costs from the workspace (layout of carve() in mtg_tube_time.hip:
    // coeffs, pts, qcost, ... each 256-byte aligned) while it is still owned.
    const int P = grad_mode == 2 ? 9 : 1;
    auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t o_pts = up(sizeof(double) * P * 4 * 3 * 10);
    const size_t o_qc = up(o_pts + sizeof(double) * P * 4);
    std::vector<double> pts(P * 4), qc(P);
    HIP_OK(hipMemcpy(pts.data(), static_cast<char*>(ws) + o_pts, pts.size() * 8,
                     hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(qc.data(), static_cast<char*>(ws) + o_qc, qc.size() * 8,
                     hipMemcpyDeviceToHost));
    r.pts_ok = true;
    for (int j = 0; j < P; ++j)
      for (int i = 0; i < 4; ++i) {
        double e = t[i];
        if (j > 0 && i == (j - 1) / 2) e = (j & 1) ? e - 0.1 : e + 0.1;
        if (pts[j * 4 + i] != e) r.pts_ok = false;
      }
    r.qcost0 = qc[0];
    r.pts0 = pts[0];
  }
  if (pooled && mode != "pool") HIP_OK(hipFreeAsync(ws, s));
  if (!pooled) HIP_OK(hipFree(ws));
  if (s) HIP_OK(hipStreamDestroy(s));
  r.g.resize(4);
  HIP_OK(hipMemcpy(&r.J, cost, sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(r.g.data(), grad, 4 * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&r.st, st, sizeof(int32_t), hipMemcpyDeviceToHost));
  for (void* q : {static_cast<void*>(pos), static_cast<void*>(df), static_cast<void*>(tcp),
                  static_cast<void*>(tt), static_cast<void*>(rad), static_cast<void*>(cost),
                  static_cast<void*>(grad), static_cast<void*>(st)})
    HIP_OK(hipFree(q));
  return r;
}

bool same(const Result& a, const Result& b, int grad_mode) {
  if (std::memcmp(&a.J, &b.J, sizeof(double)) != 0 || a.st != b.st) return false;
  if (grad_mode) return std::memcmp(a.g.data(), b.g.data(), 4 * sizeof(double)) == 0;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 30;
  mtg_ctx* ctx = nullptr;
  if (mtg_ctx_create(0, &ctx) != MTG_OK) return 5;
  const Inputs in = mainCpp();
  std::vector<double> t = in.t0;
  for (double& v : t) v *= 1.05;
  struct Call {
    const char* name;
    const std::vector<double>* t;
    int grad;
  } calls[3] = {{"J(1.05T),grad", &t, 2}, {"J(T0)", &in.t0, 0}, {"J(T0),grad", &in.t0, 2}};
  Result ref[3];
  for (int c = 0; c < 3; ++c) ref[c] = evaluate(ctx, in, *calls[c].t, calls[c].grad, "plain");
  for (int c = 0; c < 3; ++c)
    std::printf("reference %-14s J %.17g status %d\n", calls[c].name, ref[c].J, ref[c].st);
  int bad_total = 0;
  for (const char* mode : {"pool_sync", "pool_stream", "plain"}) {
    int mism = 0, nan = 0, stale = 0, unwritten = 0, overl = 0, overl_mism = 0;
    for (int it = 0; it < reps; ++it)
      for (int c = 0; c < 3; ++c) {
        const Result r = evaluate(ctx, in, *calls[c].t, calls[c].grad, mode);
        if (r.overlap) ++overl;
        if (same(r, ref[c], calls[c].grad)) continue;
        if (r.overlap) ++overl_mism;
        ++mism;
        if (std::isnan(r.J)) ++nan;
        if (r.J == 12345.0) ++unwritten;
        for (int o = 0; o < 3; ++o)
          if (o != c && r.J == ref[o].J) ++stale;
        if (mism <= 8)
          std::printf("  %s it %d %-14s J %.17g status %d (expected %.17g), workspace "
                      "overlaps %d live buffer(s); points intact %d (T0 %.17g), QCQP cost %.17g\n",
                      mode, it, calls[c].name, r.J, r.st, ref[c].J, r.overlap, r.pts_ok ? 1 : 0,
                      r.pts0, r.qcost0);
      }
    std::printf("mode %-11s: %d calls, %d mismatches (NaN %d, equal to another call's J %d, "
                "never written %d); workspace overlapped a live buffer in %d calls, %d of "
                "them mismatched\n",
                mode, 3 * reps, mism, nan, stale, unwritten, overl, overl_mism);
    bad_total += mism;
  }
  mtg_ctx_destroy(ctx);
  return bad_total ? 1 : 0;
}
