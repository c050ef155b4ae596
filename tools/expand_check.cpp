/* expand_check.cpp -- CPU check that the engine's parallel descriptor
   expansion (expand_par) equals the serial one (expand) byte for byte, on
   random transaction batches with and without the block-count grouping, and
   fails the same way on out-of-bounds descriptors and max_sig overflows.
   Built and run by tests/test_expand_par.py (no GPU needed):
     hipcc -O2 -std=c++17 -x hip tools/expand_check.cpp -o build/expand_check \
           -L firedancer_amd -l:libfd_ed25519_gpu.so -Wl,-rpath,$PWD/firedancer_amd */
#include "../firedancer_amd/csrc/fdgpu_engine.cpp"

#include <random>

int main() {
  std::mt19937_64 rng(0xE4);
  int bad = 0;
  for (int trial = 0; trial < 24; trial++) {
    const uint64_t n = 65536 + (rng() % 200000), arena = 1ull << 26;
    std::vector<fdgpu_txn_t> tx(n);
    for (auto &x : tx) {
      x.sig_cnt = (uint32_t)(rng() % 20 == 0 ? rng() % 20 : 1 + rng() % 12);   /* some 0 / >16: skipped */
      x.msg_sz = (uint32_t)(rng() % 1300);
      x.msg_off = (uint32_t)(rng() % (arena - 2048));
      x.sig_off = (uint32_t)(rng() % (arena - 2048));
      x.pub_off = (uint32_t)(rng() % (arena - 2048));
    }
    uint64_t max_sig = n * 16;
    const int mode = trial % 4;          /* 0, 1: valid; 2: a bad descriptor; 3: max_sig overflow */
    if (mode == 2) tx[rng() % n].msg_off = (uint32_t)arena;
    if (mode == 3) { max_sig = n * 3; if (trial & 4) tx[rng() % n].pub_off = (uint32_t)arena; }   /* whichever comes first */
    for (int grouped = 0; grouped < 2; grouped++) {
      std::vector<fdgpu_sig_desc_t> s1(max_sig + 16), s2(max_sig + 16);
      std::vector<fdgpu_txn_desc_t> t1(n), t2(n);
      std::vector<uint32_t> p1(max_sig + 16), p2(max_sig + 16);
      const int64_t a = expand(arena, tx.data(), n, max_sig, s1.data(), t1.data(), grouped ? p1.data() : nullptr);
      const std::string e1 = g_err;
      const int64_t b = expand_par(arena, tx.data(), n, max_sig, s2.data(), t2.data(), grouped ? p2.data() : nullptr);
      const std::string e2 = g_err;
      bool ok = a == b;
      if (ok && a < 0) ok = e1 == e2;
      if (ok && a >= 0) {
        ok = !memcmp(s1.data(), s2.data(), (size_t)a * sizeof(fdgpu_sig_desc_t)) &&
             !memcmp(t1.data(), t2.data(), n * sizeof(fdgpu_txn_desc_t)) &&
             (!grouped || !memcmp(p1.data(), p2.data(), (size_t)a * sizeof(uint32_t)));
      }
      printf("trial %d mode %d grouped %d: n %llu -> %lld / %lld %s%s\n", trial, mode, grouped, (unsigned long long)n,
             (long long)a, (long long)b, ok ? "equal" : "DIFFER", a < 0 ? (" (" + e1 + ")").c_str() : "");
      bad += !ok;
    }
  }
  printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}
