// Host-side sanitizer driver for the native GEMM planner / tuning table.
// Built by tests/test_native_sanitizers.py with ASan+UBSan (and separately TSan) on the HOST
// side only (-Xarch_host), linked against ops/csrc/gemm.hip + gemm_areg.hip with the tile
// launchers stubbed out -- nothing here touches a GPU.  It exercises what serving exercises:
// the generation thread and the scorer thread planning GEMMs concurrently while the tuning
// table is loaded / cleared, and checks that planning is deterministic.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"

// the tile launchers of the other translation units: never reached (no launch happens here)
void gemm_c0_buf_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_c0_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_c1_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_c2_buf_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_c2_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_c3_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_pp_c0_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
void gemm_pp_c2_launch(const GemmArgs&, float*, hipStream_t) { std::abort(); }
bool launch_gemv(const GemmArgs&, hipStream_t) { std::abort(); }

static std::vector<GemmArgs> shapes() {
  std::vector<GemmArgs> v;
  const int mnk[][3] = {{32768, 320, 320}, {32768, 960, 320}, {32768, 1280, 320}, {8192, 640, 640},
                        {8192, 1920, 640}, {2048, 1280, 1280}, {512, 1280, 11520}, {77, 768, 768},
                        {4096, 4096, 4096}, {33, 5, 8}, {1, 320, 1280}};
  static uint16_t dummy[64] __attribute__((aligned(64)));
  for (auto& s : mnk)
    for (int act : {0, 2, 4}) {
      GemmArgs p;
      p.A = dummy; p.W = dummy; p.C = dummy;
      p.M = s[0]; p.N = s[1]; p.K = s[2];
      p.Nw = act == 4 ? 2 * s[1] : s[1];
      p.lda = p.K; p.ldc = p.N; p.act = act;
      v.push_back(p);
    }
  return v;
}

int main() {
  const auto sh = shapes();
  std::vector<GemmPlan> ref;
  for (auto& p : sh) ref.push_back(gemm_plan(p));
  std::vector<std::string> keys;
  for (auto& p : sh) keys.push_back(gemm_key(p));
  int bad = 0;
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int it = 0; it < 200; ++it)
        for (size_t i = 0; i < sh.size(); ++i) {
          const GemmPlan g = gemm_plan(sh[i]);
          if (gemm_key(sh[i]) != keys[i]) __atomic_add_fetch(&bad, 1, __ATOMIC_RELAXED);
          (void)g;
          int c, s;
          gemm_last_plan(&c, &s);
          if (c != g.cfg || s != g.split) __atomic_add_fetch(&bad, 1, __ATOMIC_RELAXED);
        }
      (void)t;
    });
  for (int it = 0; it < 200; ++it) {          // a table being (re)loaded meanwhile
    for (size_t i = 0; i < sh.size(); i += 3) gemm_tune_set(keys[i], ref[i].cfg, ref[i].split);
    (void)gemm_tune_size();
    gemm_tune_clear();
  }
  for (auto& x : th) x.join();
  for (size_t i = 0; i < sh.size(); ++i) {
    const GemmPlan g = gemm_plan(sh[i]);
    if (g.cfg != ref[i].cfg || g.split != ref[i].split) ++bad;
  }
  std::printf("planner shapes %zu, mismatches %d\n", sh.size(), bad);
  return bad ? 1 : 0;
}
