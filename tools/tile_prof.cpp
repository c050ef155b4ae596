/* tile_prof.cpp -- host-side cost probe of the verify mux tile, no GPU: the
   tile (fdgpu_vmux on fdt_mux_run) drains a prefilled quic->verify link of
   real payloads through the null verifier (tools/null_verifier.c), while a
   SIGPROF timer on the tile thread samples its program counter; samples are
   mapped to symbols of the loaded objects.  Bench infrastructure only.

     g++ -O2 -g -std=c++17 -I include tools/tile_prof.cpp tools/null_verifier.c -o tools/tile_prof \
         -L firedancer_amd -l:libfd_verify_tile.so -Wl,-rpath,$PWD/firedancer_amd -lpthread -ldl
     tools/tile_prof <payloads.bin> <offs.bin> <sizes.bin> [gpu_parse 0|1|2] [repeat]

   (payload files: numpy tofile of workload.pack_payloads' arena / offs u64 /
   sizes u32.) */
#define _GNU_SOURCE 1
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

extern "C" {
#include "fd_verify_tile.h"
void null_verifier_make(fdgpu_verifier_t *out);
}

static uint64_t now_ns() { timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec * 1000000000ull + ts.tv_nsec; }

template <class T> static std::vector<T> rd(const char *p) {
  FILE *f = fopen(p, "rb");
  if (!f) { perror(p); exit(1); }
  fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (fread(v.data(), 1, n, f) != (size_t)n) exit(1);
  fclose(f);
  return v;
}

static std::vector<void *> g_pcs;
static std::atomic<bool> g_on{false};
static void on_prof(int, siginfo_t *, void *uc) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const ucontext_t *u = (const ucontext_t *)uc;
  if (g_pcs.size() < g_pcs.capacity()) g_pcs.push_back((void *)u->uc_mcontext.gregs[REG_RIP]);
}

int main(int argc, char **argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s payloads offs sizes [gpu_parse] [repeat]\n", argv[0]); return 2; }
  auto A = rd<uint8_t>(argv[1]);
  auto O = rd<uint64_t>(argv[2]);
  auto S = rd<uint32_t>(argv[3]);
  const int gpu_parse = argc > 4 ? atoi(argv[4]) : 1;
  const int repeat = argc > 5 ? atoi(argv[5]) : 3;
  const int tiles = getenv("TILE_PROF_TILES") ? atoi(getenv("TILE_PROF_TILES")) : 1;
  const uint64_t n = O.size(), depth = 1ull << 21;
  /* in link: mcache + dcache, prefilled */
  std::vector<fdt_frag_meta_t> in_mc(depth);
  const uint64_t in_data = fdt_dcache_data_sz(FDT_TPU_MTU, depth);
  std::vector<uint8_t> in_dc(in_data + 64);
  uint8_t *in_base = (uint8_t *)(((uintptr_t)in_dc.data() + 63) & ~(uintptr_t)63);
  const uint64_t in_chunk0 = 0, in_wmark = fdt_dcache_wmark(0, in_data / 64, FDT_TPU_MTU);
  /* out link */
  const uint64_t out_depth = 1ull << 14, batch = 16384, inflight = 4;
  const uint64_t out_data = fdgpu_vmux_dcache_data_sz(out_depth, (uint32_t)batch, (uint32_t)inflight);
  std::vector<std::vector<fdt_frag_meta_t>> out_mcs(tiles, std::vector<fdt_frag_meta_t>(out_depth));
  std::vector<std::vector<uint8_t>> out_dcs(tiles, std::vector<uint8_t>(out_data + 64));
  std::vector<fdgpu_verifier_t> vers(tiles);
  for (auto &v : vers) null_verifier_make(&v);
  struct sigaction sa{};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  g_pcs.reserve(1 << 22);
  double best = 1e30;
  for (int r = 0; r < repeat; r++) {
    fdt_mcache_init(in_mc.data(), depth, 0);
    uint64_t chunk = in_chunk0;
    for (uint64_t i = 0; i < n; i++) {
      memcpy(in_base + (chunk << 6), A.data() + O[i], S[i]);
      fdt_mcache_publish(in_mc.data(), depth, i, 0, chunk, S[i], fdt_frag_meta_ctl(0, 1, 1, 0), 0, 0);
      chunk = fdt_dcache_compact_next(chunk, S[i], in_chunk0, in_wmark);
    }
    std::vector<fdgpu_vmux_t *> vms(tiles);
    std::vector<fdt_mux_cfg_t> mcs(tiles);
    std::vector<uint64_t> halts(tiles, 0);        /* read by fdt_mux_run through a volatile pointer */
    std::vector<fdt_mux_stats_t> mss(tiles);
    fdt_mux_callbacks_t cb = fdgpu_vmux_callbacks();
    for (int k = 0; k < tiles; k++) {
      fdt_mcache_init(out_mcs[k].data(), out_depth, 0);
      uint8_t *out_base = (uint8_t *)(((uintptr_t)out_dcs[k].data() + 63) & ~(uintptr_t)63);
      fdgpu_vmux_cfg_t vc{};
      vc.in_cnt = 1; vc.in_base[0] = in_base; vc.in_chunk0[0] = in_chunk0; vc.in_wmark[0] = in_wmark;
      vc.out_base = out_base; vc.out_chunk0 = 0; vc.out_wmark = fdt_dcache_wmark(0, out_data / 64, FDT_TPU_DCACHE_MTU);
      vc.cr_max = out_depth; vc.round_robin_idx = (uint64_t)k; vc.round_robin_cnt = (uint64_t)tiles; vc.hashmap_seed = 0x5EED;
      vc.batch_txn_max = (uint32_t)batch; vc.inflight_max = (uint32_t)inflight; vc.batch_wait_ns = 200000;
      vc.batch_bytes_max = batch * 2176; vc.gpu_parse = (uint32_t)gpu_parse;
      vc.in_mcache[0] = in_mc.data(); vc.in_depth[0] = depth;
      vms[k] = fdgpu_vmux_new(&vc, vers[k]);
      if (!vms[k]) { fprintf(stderr, "vmux_new failed\n"); return 1; }
      fdt_mux_cfg_t &mc = mcs[k];
      mc = fdt_mux_cfg_t{};
      mc.in_cnt = 1; mc.in_mcache[0] = in_mc.data(); mc.in_depth[0] = depth; mc.in_seq0[0] = 0;
      mc.out_mcache = out_mcs[k].data(); mc.out_depth = out_depth; mc.out_seq0 = 0;
      mc.flags = FDT_MUX_FLAG_COPY | FDT_MUX_FLAG_MANUAL_PUBLISH; mc.burst = 1; mc.cr_max = out_depth; mc.lazy_iters = 16;
    }
    pid_t tid = 0;
    std::atomic<int> started{0};
    uint64_t t0 = 0;
    std::vector<std::thread> ths;
    for (int k = 0; k < tiles; k++)
      ths.emplace_back([&, k]() {
        if (getenv("TILE_PROF_CPU")) {                  /* tile k alone on CPU base + k */
          cpu_set_t cs; CPU_ZERO(&cs); CPU_SET(atoi(getenv("TILE_PROF_CPU")) + k, &cs);
          pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
        }
        if (k == 0) { tid = (pid_t)syscall(SYS_gettid); t0 = now_ns(); }
        started++;
        while (started.load() < tiles) {}
        fdt_mux_run(&mcs[k], &cb, vms[k], (volatile uint64_t *)&halts[k], &mss[k]);
      });
    while (started.load() < tiles || !tid) {}
    timer_t tm;
    sigevent se{};
    se.sigev_notify = SIGEV_THREAD_ID;
    se._sigev_un._tid = tid;
    se.sigev_signo = SIGPROF;
    timer_create(CLOCK_MONOTONIC, &se, &tm);
    itimerspec its{};
    its.it_interval.tv_nsec = its.it_value.tv_nsec = getenv("TILE_PROF_OFF") ? 0 : 200000;   /* 5 kHz (tile 0) */
    g_on = true;
    timer_settime(tm, 0, &its, nullptr);
    for (int k = 0; k < tiles; k++)
      while (fdgpu_vmux_final_cnt(vms[k]) < n) usleep(20);   /* never on a tile's CPU for long */
    const uint64_t t1 = now_ns();
    g_on = false;
    for (int k = 0; k < tiles; k++) __atomic_store_n(&halts[k], 1, __ATOMIC_RELEASE);
    for (auto &th : ths) th.join();
    timer_delete(tm);
    uint64_t pub = 0, pf = 0;
    for (int k = 0; k < tiles; k++) {
      fdgpu_vtile_stats_t st;
      fdgpu_vmux_stats(vms[k], &st);
      pub += st.published; pf += st.parse_fail;
    }
    const double ns = (double)(t1 - t0) / n;
    best = std::min(best, ns);
    printf("run %d (%d tiles): %.1f ns/frag (%.2f M/s)  published %llu parse_fail %llu\n", r, tiles, ns, 1e3 / ns,
           (unsigned long long)pub, (unsigned long long)pf);
    for (int k = 0; k < tiles; k++) fdgpu_vmux_delete(vms[k]);
  }
  /* symbolise: object + offset (for addr2line -f -i -e <object>) */
  std::map<std::string, uint64_t> by;
  FILE *raw = getenv("TILE_PROF_RAW") ? fopen(getenv("TILE_PROF_RAW"), "w") : nullptr;
  for (void *pc : g_pcs) {
    Dl_info di;
    std::string name = "?";
    if (dladdr(pc, &di) && di.dli_sname) name = di.dli_sname;
    else if (dladdr(pc, &di) && di.dli_fname) name = std::string("[") + di.dli_fname + "]";
    if (raw && dladdr(pc, &di) && di.dli_fname)
      fprintf(raw, "%s 0x%lx\n", di.dli_fname, (unsigned long)((uintptr_t)pc - (uintptr_t)di.dli_fbase));
    by[name]++;
  }
  if (raw) fclose(raw);
  std::vector<std::pair<uint64_t, std::string>> v;
  for (auto &kv : by) v.push_back({kv.second, kv.first});
  std::sort(v.rbegin(), v.rend());
  printf("best %.1f ns/frag; %zu samples\n", best, g_pcs.size());
  for (size_t i = 0; i < v.size() && i < 25; i++) printf("  %5.1f%%  %s\n", 100.0 * v[i].first / g_pcs.size(), v[i].second.c_str());
  return 0;
}
