/* fdt_sandbox.cpp -- process separation for the verify stage (SURVEY.md
   §8(f) row 1, last bullet): tango links laid out in one shared-memory
   region that independent processes join, and the tiles' seccomp sandbox.

   Why: the reference's tiles run one per process and, after privileged init,
   inside a seccomp policy that allows only write(2 or logfile_fd) and
   fsync(logfile_fd) (src/app/fdctl/run/tiles/verify.seccomppolicy:1-19,
   dedup.seccomppolicy; entered at src/disco/topo/fd_topo_run.c:96-103).  A
   GPU engine needs ioctls on /dev/kfd for every submission, so the GPU side
   runs as its own (unsandboxed) engine process, fed over tango links in
   shared memory -- the wiredancer precedent (src/wiredancer/c/wd_f1.h:71-112)
   -- while the tiles around it (dedup, and anything else that only touches
   links) keep the reference's sandbox.

   Link region layout (fdt_link_new / fdt_link_join; offsets from the region
   base, every part 4 KiB aligned so the region can be mapped anywhere):
     [0, 4096)        header: magic, depth, mtu, seq0, data_sz, mcache_off,
                      dcache_off; the consumer fseq on its own 128-B line
     [4096, ...)      mcache: depth x fdt_frag_meta_t (fd_mcache.h:265-322)
     [dcache_off, ..) compact dcache for depth frags of <= mtu (fd_dcache.h) */
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sched.h>
#include <signal.h>
#include <ucontext.h>
#include <linux/audit.h>
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <stddef.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "../../../include/fd_verify_tile.h"

namespace {

constexpr uint64_t LINK_MAGIC = 0xFD7A960114C0DE01ull;
constexpr uint64_t LINK_HDR = 4096;
constexpr uint64_t FSEQ_OFF = 128;

struct link_hdr {
  uint64_t magic, depth, mtu, seq0, data_sz, mcache_off, dcache_off;
};

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

}  // namespace

extern "C" {

uint64_t fdt_link_footprint_sz(uint64_t depth, uint64_t mtu, uint64_t data_sz) {
  if (!depth || (depth & (depth - 1)) || !mtu) return 0;
  if (!data_sz) data_sz = fdt_dcache_data_sz(mtu, depth);
  data_sz = align_up(data_sz, FDT_CHUNK_SZ);
  if (data_sz < 2 * align_up(mtu, FDT_CHUNK_SZ)) return 0;       /* the compact ring holds two frags */
  const uint64_t dc_off = align_up(LINK_HDR + depth * sizeof(fdt_frag_meta_t), 4096);
  return align_up(dc_off + data_sz, 4096);
}

uint64_t fdt_link_footprint(uint64_t depth, uint64_t mtu) { return fdt_link_footprint_sz(depth, mtu, 0); }

int fdt_link_new_sz(void *mem, uint64_t depth, uint64_t mtu, uint64_t seq0, uint64_t data_sz) {
  const uint64_t fp = fdt_link_footprint_sz(depth, mtu, data_sz);
  if (!mem || !fp || ((uintptr_t)mem & 4095)) return -1;
  auto *h = (link_hdr *)mem;
  h->magic = 0;                                   /* not joinable until fully formatted */
  h->depth = depth;
  h->mtu = mtu;
  h->seq0 = seq0;
  h->data_sz = align_up(data_sz ? data_sz : fdt_dcache_data_sz(mtu, depth), FDT_CHUNK_SZ);
  h->mcache_off = LINK_HDR;
  h->dcache_off = align_up(LINK_HDR + depth * sizeof(fdt_frag_meta_t), 4096);
  *(volatile uint64_t *)((uint8_t *)mem + FSEQ_OFF) = seq0;
  fdt_mcache_init((fdt_frag_meta_t *)((uint8_t *)mem + h->mcache_off), depth, seq0);
  __atomic_store_n(&h->magic, LINK_MAGIC, __ATOMIC_RELEASE);
  return 0;
}

int fdt_link_new(void *mem, uint64_t depth, uint64_t mtu, uint64_t seq0) { return fdt_link_new_sz(mem, depth, mtu, seq0, 0); }

int fdt_link_join(void *mem, fdt_link_t *out) {
  if (!mem || !out) return -1;
  auto *h = (link_hdr *)mem;
  if (__atomic_load_n(&h->magic, __ATOMIC_ACQUIRE) != LINK_MAGIC) return -1;
  auto *base = (uint8_t *)mem;
  out->mcache = (fdt_frag_meta_t *)(base + h->mcache_off);
  out->depth = h->depth;
  out->seq0 = h->seq0;
  out->mtu = h->mtu;
  out->base = base + h->dcache_off;
  out->chunk0 = 0;
  out->wmark = fdt_dcache_wmark(0, h->data_sz >> FDT_CHUNK_LG_SZ, h->mtu);
  out->fseq = (uint64_t *)(base + FSEQ_OFF);
  return 0;
}

/* The tiles' policy, restated as a classic-BPF seccomp filter:
     write   iff fd == 2 or fd == logfile_fd   (verify.seccomppolicy:11-12)
     fsync   iff fd == logfile_fd              (:17)
     exit, exit_group                          (leaving the loop)
     clock_gettime                             (only reached when the vDSO
                                                falls back to the syscall)
   anything else kills the process (SECCOMP_RET_KILL_PROCESS), as the
   reference's generated filters do. */
int fdt_sandbox_enter(int logfile_fd) {
  const uint32_t lfd = (uint32_t)(logfile_fd < 0 ? 2 : logfile_fd);
  struct sock_filter f[] = {
    BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, arch)),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, 1, 0),
    BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS),
    BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, nr)),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, __NR_write, 0, 4),
    /* write: fd in {2, logfile_fd} */
    BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0])),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, 2, 10, 0),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, lfd, 9, 0),
    BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, __NR_fsync, 0, 3),
    /* fsync: fd == logfile_fd */
    BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0])),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, lfd, 5, 0),
    BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, __NR_exit_group, 3, 0),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, __NR_exit, 2, 0),
    BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, __NR_clock_gettime, 1, 0),
    BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS),
    BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW),
  };
  struct sock_fprog prog = {(unsigned short)(sizeof(f) / sizeof(f[0])), f};
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0)) return -errno;
  if (syscall(__NR_seccomp, SECCOMP_SET_MODE_FILTER, 0, &prog)) return -errno;
  return 0;
}

/* ------------------------------------------------- engine process policy

   The GPU engine process cannot run under the tiles' write/fsync policy: every
   submission and completion of the HIP runtime is an ioctl on the device's
   file descriptors, its worker threads wait on futexes and the runtime maps
   and unmaps memory as it runs.  What it never needs once its engines are
   open, warmed and registered is a NEW resource from outside the process:
   no open, socket, exec, fork, ptrace, mount, kill of another process.  So
   the engine process enters (after privileged init, as fd_topo_run.c:96-103
   enters the tiles' policies) a policy that allows the resource-neutral
   syscalls below, ioctl only on the device fds it already holds, clone only
   for threads, tgkill only to its own threads -- and kills the process on anything else, for every thread
   (SECCOMP_FILTER_FLAG_TSYNC: the runtime's threads included).

   Report mode (bring-up and tests): a syscall outside the list is refused
   all the same -- it fails with EPERM instead of killing the process, and
   is recorded (fdt_sandbox_report), so one run lists everything the
   policy refused.  Nothing outside the list is ever carried out. */

namespace {

uint64_t g_refused_bits[8];        /* syscalls < 512 refused (report mode) */
uint64_t g_refused_cnt;

void report_sigsys(int, siginfo_t *si, void *uc_) {
  const long nr = si->si_syscall;
  /* "fdt_sandbox: refused syscall <nr>" on fd 2 (write is allowed and
     async-signal-safe): calls made after the last report read, e.g. at exit */
  char msg[48] = "fdt_sandbox: refused syscall ";
  int o = 29;
  char dig[12];
  int nd = 0;
  for (long v = nr < 0 ? 0 : nr; nd == 0 || v; v /= 10) dig[nd++] = (char)('0' + v % 10);
  while (nd) msg[o++] = dig[--nd];
  msg[o++] = '\n';
  (void)!write(2, msg, (size_t)o);
  if (nr >= 0 && nr < 512) __atomic_fetch_or(&g_refused_bits[nr >> 6], 1ull << (nr & 63), __ATOMIC_RELAXED);
  __atomic_fetch_add(&g_refused_cnt, 1, __ATOMIC_RELAXED);
  ((ucontext_t *)uc_)->uc_mcontext.gregs[REG_RAX] = -EPERM;     /* the call fails; it was not made */
}

/* the syscalls of a running engine process (the HIP runtime's submissions,
   waits and memory management, the tiles' clocks and yields, the Python
   loop around them), none of which reaches outside the process */
const uint32_t ENGINE_ALLOW[] = {
  __NR_read, __NR_write, __NR_pread64, __NR_pwrite64, __NR_readv, __NR_writev, __NR_lseek, __NR_fstat,
  __NR_close, __NR_fsync, __NR_fdatasync, __NR_dup, __NR_fcntl,
  __NR_mmap, __NR_munmap, __NR_mprotect, __NR_mremap, __NR_madvise, __NR_brk, __NR_mlock, __NR_munlock,
  __NR_futex, __NR_sched_yield, __NR_nanosleep, __NR_clock_nanosleep, __NR_clock_gettime, __NR_clock_getres,
  __NR_gettimeofday, __NR_select, __NR_pselect6, __NR_poll, __NR_ppoll, __NR_epoll_wait, __NR_epoll_pwait,
  __NR_getpid, __NR_gettid, __NR_getppid, __NR_getuid, __NR_geteuid, __NR_getgid, __NR_getegid,
  __NR_rt_sigprocmask, __NR_rt_sigaction, __NR_rt_sigreturn, __NR_sigaltstack,
  __NR_sched_getaffinity, __NR_sched_setaffinity, __NR_sched_getparam, __NR_sched_getscheduler,
  __NR_set_robust_list, __NR_rseq, __NR_getrandom, __NR_membarrier, __NR_getrusage,
  __NR_mbind, __NR_get_mempolicy,                     /* the HIP runtime's NUMA placement of host memory */
  __NR_exit, __NR_exit_group,
};

}  // namespace

int fdt_sandbox_driver_fds(int *out, int max) {
  DIR *d = opendir("/proc/self/fd");
  if (!d) return -errno;
  const int self = dirfd(d);
  int n = 0;
  for (struct dirent *e; (e = readdir(d));) {
    char *end = nullptr;
    const long fd = strtol(e->d_name, &end, 10);
    if (!e->d_name[0] || *end || fd == self) continue;
    char link[64], target[256];
    snprintf(link, sizeof link, "/proc/self/fd/%ld", fd);
    const ssize_t k = readlink(link, target, sizeof target - 1);
    if (k <= 0) continue;
    target[k] = 0;
    if (strcmp(target, "/dev/kfd") && strncmp(target, "/dev/dri/", 9)) continue;
    if (n < max) out[n] = (int)fd;
    n++;
  }
  closedir(d);
  if (n > max) return -ENOSPC;
  std::sort(out, out + n);
  return n;
}

int fdt_sandbox_engine_enter(const int *dev_fds, int dev_fd_cnt, int report) {
  if (dev_fd_cnt < 0 || dev_fd_cnt > 64 || (dev_fd_cnt && !dev_fds)) return -EINVAL;
  const uint32_t KILL = SECCOMP_RET_KILL_PROCESS, ALLOW = SECCOMP_RET_ALLOW;
  const uint32_t DENY = report ? SECCOMP_RET_TRAP : KILL;
  std::vector<sock_filter> f;
  auto stmt = [&](uint16_t code, uint32_t k) { f.push_back(BPF_STMT(code, k)); };
  auto jeq = [&](uint32_t k, uint8_t jt, uint8_t jf) { f.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, k, jt, jf)); };
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, arch));
  jeq(AUDIT_ARCH_X86_64, 1, 0);
  stmt(BPF_RET | BPF_K, KILL);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, nr));
  for (uint32_t nr : ENGINE_ALLOW) {
    jeq(nr, 0, 1);
    stmt(BPF_RET | BPF_K, ALLOW);
  }
  /* clone: threads only (CLONE_THREAD in the flags, arg 0); clone3: ENOSYS,
     so the C library falls back to clone, whose flags the filter can read */
  jeq(__NR_clone3, 0, 1);
  stmt(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | ENOSYS);
  jeq(__NR_clone, 0, 4);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0]));
  f.push_back(BPF_JUMP(BPF_JMP | BPF_JSET | BPF_K, CLONE_THREAD, 0, 1));
  stmt(BPF_RET | BPF_K, ALLOW);
  stmt(BPF_RET | BPF_K, DENY);
  /* tgkill: signals to this process's own threads only (thread group = our
     pid: raise, abort, pthread_kill); a signal to any other process is refused */
  jeq(__NR_tgkill, 0, 4);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0]));
  jeq((uint32_t)getpid(), 0, 1);
  stmt(BPF_RET | BPF_K, ALLOW);
  stmt(BPF_RET | BPF_K, DENY);
  /* newfstatat: the fstat form only (AT_EMPTY_PATH, as the C library's
     fstat issues it).  The flag does not stop a non-empty path from being
     looked up, and the filter cannot read the string: such a call can read a
     path's metadata, but it opens nothing and yields no fd */
  jeq(__NR_newfstatat, 0, 4);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[3]));
  f.push_back(BPF_JUMP(BPF_JMP | BPF_JSET | BPF_K, AT_EMPTY_PATH, 0, 1));
  stmt(BPF_RET | BPF_K, ALLOW);
  stmt(BPF_RET | BPF_K, DENY);
  /* prctl: thread names only (PR_SET_NAME / PR_GET_NAME), not the options
     that would open the process to others (PR_SET_PTRACER, _DUMPABLE) */
  jeq(__NR_prctl, 0, 5);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0]));
  jeq(PR_SET_NAME, 1, 0);
  jeq(PR_GET_NAME, 0, 1);
  stmt(BPF_RET | BPF_K, ALLOW);
  stmt(BPF_RET | BPF_K, DENY);
  /* prlimit64: reading this process's own limits only (pid 0, no new
     limit: the HIP runtime's teardown asks) */
  jeq(__NR_prlimit64, 0, 8);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0]));
  jeq(0, 0, 4);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[2]));
  jeq(0, 0, 2);
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[2]) + 4);
  jeq(0, 1, 0);
  stmt(BPF_RET | BPF_K, DENY);
  stmt(BPF_RET | BPF_K, ALLOW);
  /* ioctl: only on the device fds held at entry (/dev/kfd, the render nodes) */
  jeq(__NR_ioctl, 0, (uint8_t)(2 + 2 * dev_fd_cnt));
  stmt(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, args[0]));
  for (int i = 0; i < dev_fd_cnt; i++) {
    jeq((uint32_t)dev_fds[i], 0, 1);
    stmt(BPF_RET | BPF_K, ALLOW);
  }
  stmt(BPF_RET | BPF_K, DENY);
  stmt(BPF_RET | BPF_K, DENY);
  if (f.size() > 4096) return -E2BIG;
  if (report) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = report_sigsys;
    sa.sa_flags = SA_SIGINFO | SA_NODEFER;
    if (sigaction(SIGSYS, &sa, nullptr)) return -errno;
  }
  struct sock_fprog prog = {(unsigned short)f.size(), f.data()};
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0)) return -errno;
  if (syscall(__NR_seccomp, SECCOMP_SET_MODE_FILTER, SECCOMP_FILTER_FLAG_TSYNC, &prog)) return -errno;
  return 0;
}

uint64_t fdt_sandbox_report(uint64_t *bits8) {
  for (int i = 0; i < 8; i++) bits8[i] = __atomic_load_n(&g_refused_bits[i], __ATOMIC_RELAXED);
  return __atomic_load_n(&g_refused_cnt, __ATOMIC_RELAXED);
}

/* Dedup tile main loop inside the sandbox (a child process of whoever set
   up the links): steps until frag_target frags were consumed or nothing
   arrived for idle_ns_max, stores the final stats into stats_out (shared
   memory the parent reads) and exits the process: 0 target reached, 1 idle
   timeout, 3 sandbox could not be entered.  Never returns. */
void fdgpu_dtile_run_sandboxed(fdgpu_dtile_t *t, uint64_t frag_target, uint64_t idle_ns_max,
                               fdgpu_dtile_stats_t *stats_out, int logfile_fd) {
  if (fdgpu_dtile_rehome(t) || fdt_sandbox_enter(logfile_fd)) syscall(__NR_exit_group, 3);
  fdgpu_dtile_stats_t st;
  uint64_t last = mono_ns(), last_frag = 0;
  int rc = 0;
  /* the clock is read only on idle passes, every 256th: a pass that took a
     frag costs no clock read and no stats copy beyond the step itself */
  for (uint64_t idle = 0;;) {                          /* 64-bit: never wraps back to the first check */
    if (fdgpu_dtile_step(t) > 0) {
      idle = 0;
      fdgpu_dtile_stats(t, &st);
      if (st.in_frags + st.overrun >= frag_target) { last_frag = mono_ns(); break; }
      continue;
    }
    if ((++idle & 255u) == 0) {
      const uint64_t now = mono_ns();
      if (idle == 256u) last = last_frag = now;         /* the first idle check since the last frag */
      fdgpu_dtile_stats(t, &st);
      if (st.in_frags + st.overrun >= frag_target) break;
      if (now - last > idle_ns_max) { rc = 1; break; }
    }
  }
  st.done_ns = st.in_frags ? last_frag : 0;
  memcpy(stats_out, &st, sizeof(st));
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  syscall(__NR_exit_group, rc);
  for (;;) {}
}

}  // extern "C"
