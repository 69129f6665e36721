// kb_xfer.h — the cross-shard exchange of the sharded simulator, host side.
//
// A mesh of C peer ids can be split into `world` contiguous row shards: rank k holds the rows (the
// observer state) of ids [k*S, min(C, (k+1)*S)), S = ceil(C / world).  Per round the shards exchange
// exactly what the reference's UDP transport carries between instances (src/kaboodle.rs:188-226):
// the unicast records of every delivery wave with the ids of KnownPeers lists (all-to-all-v), and
// the Join / Failed broadcast lists (all-gather-v); plus two tiny reductions (agreement count, error
// flag), and the counters when asked for.
//
// Three transports implement it:
//   RcclXfer   one process per GPU: RCCL (ncclAllToAllv / ncclAllGather / ncclAllReduce) on the
//              simulator's stream, over xGMI between the MI355X devices of a node;
//   LocalXfer  the `world` shards of one mesh inside one process (one host thread and one HIP stream
//              per shard): the same exchange as device-to-device copies.  It lets the sharded code
//              path be tested bit-exact against the oracle on a single GPU;
//   IpcXfer    ranks in separate processes sharing one device (a test transport: RCCL refuses two ranks
//              on one GPU), over IPC-mapped device windows and a shared-memory rendezvous.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <string>
#include <vector>

namespace kb {

struct Xfer {
  int rank = 0, world = 1;
  virtual ~Xfer() {}
  // all-to-all-v of `elem`-byte elements between device buffers; counts and displacements are in
  // elements, indexed by peer rank (host arrays, the meaning of ncclAllToAllv's)
  virtual bool alltoallv(const void* send, const size_t* scounts, const size_t* sdispls, void* recv,
                         const size_t* rcounts, const size_t* rdispls, size_t elem, hipStream_t st) = 0;
  // every rank contributes `count` u32 from `send`; `recv` gets world*count u32 in rank order
  virtual bool allgather_u32(const uint32_t* send, uint32_t* recv, size_t count, hipStream_t st) = 0;
  // in-place reductions of small device arrays
  virtual bool allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t st) = 0;
  virtual bool allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t st) = 0;
  virtual bool allreduce_sum_u64(unsigned long long* buf, size_t count, hipStream_t st) = 0;
  virtual void abort() {}
  // brackets several exchanges that may be issued as one (RCCL group: one launch for both all-to-alls)
  virtual bool group_begin() { return true; }
  virtual bool group_end() { return true; }
  virtual std::string error() const = 0;
};

// ---- RCCL ---------------------------------------------------------------------------------------
struct RcclXfer : Xfer {
  ncclComm_t comm = nullptr;
  ncclResult_t last = ncclSuccess;
  std::vector<size_t> sc[2], sd[2], rc[2], rd[2];   // two calls can share one group: a set each
  int cur = 0;
  bool ok(ncclResult_t r) { last = r; return r == ncclSuccess; }
  bool init(int r, int w, const void* uid) {
    rank = r; world = w;
    for (int b = 0; b < 2; ++b) { sc[b].resize(w); sd[b].resize(w); rc[b].resize(w); rd[b].resize(w); }
    ncclUniqueId id;
    memcpy(&id, uid, sizeof id);
    return ok(ncclCommInitRank(&comm, w, id, r));
  }
  ~RcclXfer() override { if (comm) ncclCommDestroy(comm); }
  bool group_begin() override { return ok(ncclGroupStart()); }
  bool group_end() override { return ok(ncclGroupEnd()); }
  bool alltoallv(const void* send, const size_t* scounts, const size_t* sdispls, void* recv, const size_t* rcounts,
                 const size_t* rdispls, size_t elem, hipStream_t st) override {
    // moved as bytes: counts and displacements scale by the element size
    const int b = cur; cur ^= 1;
    for (int k = 0; k < world; ++k) {
      sc[b][k] = scounts[k] * elem; sd[b][k] = sdispls[k] * elem; rc[b][k] = rcounts[k] * elem; rd[b][k] = rdispls[k] * elem;
    }
    return ok(ncclAllToAllv(send, sc[b].data(), sd[b].data(), recv, rc[b].data(), rd[b].data(), ncclUint8, comm, st));
  }
  bool allgather_u32(const uint32_t* send, uint32_t* recv, size_t count, hipStream_t st) override {
    return ok(ncclAllGather(send, recv, count, ncclUint32, comm, st));
  }
  bool allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return ok(ncclAllReduce(buf, buf, count, ncclUint32, ncclSum, comm, st));
  }
  bool allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return ok(ncclAllReduce(buf, buf, count, ncclUint32, ncclMax, comm, st));
  }
  bool allreduce_sum_u64(unsigned long long* buf, size_t count, hipStream_t st) override {
    return ok(ncclAllReduce(buf, buf, count, ncclUint64, ncclSum, comm, st));
  }
  void abort() override { if (comm) { ncclCommAbort(comm); comm = nullptr; } }
  std::string error() const override { return std::string("RCCL: ") + ncclGetErrorString(last); }
};

// ---- in-process shards --------------------------------------------------------------------------
// Shared by the `world` shards of one mesh.  Every collective is a rendezvous: each shard drains its
// stream (its send data is then complete), publishes its pointers and waits; each shard then pulls
// what it needs from the others with device-to-device copies on its own stream, drains it, and waits
// again before anyone may reuse a send buffer.  A shard that fails aborts the hub, which releases
// every waiter with an error instead of a hang.
struct LocalHub {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<const void*> src;
  std::vector<const size_t*> sc, sd;
  std::vector<std::vector<unsigned long long>> vals;
  explicit LocalHub(int w) : world(w), src(w), sc(w), sd(w), vals(w) {}
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == world) { arrived = 0; ++gen; cv.notify_all(); return true; }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return !aborted;
  }
  void abort() { std::lock_guard<std::mutex> lk(mu); aborted = true; cv.notify_all(); }
  void reset() { std::lock_guard<std::mutex> lk(mu); aborted = false; arrived = 0; }
};

struct LocalXfer : Xfer {
  LocalHub* hub = nullptr;
  std::string err;
  bool fail(const char* what) { err = what; hub->abort(); return false; }
  void abort() override { hub->abort(); }
  bool alltoallv(const void* send, const size_t* scounts, const size_t* sdispls, void* recv, const size_t* rcounts,
                 const size_t* rdispls, size_t elem, hipStream_t st) override {
    if (hipStreamSynchronize(st) != hipSuccess) return fail("stream sync before exchange");
    hub->src[rank] = send; hub->sc[rank] = scounts; hub->sd[rank] = sdispls;
    if (!hub->barrier()) return fail("exchange aborted by another shard");
    for (int k = 0; k < world; ++k) {
      const size_t n = rcounts[k];
      if (n != hub->sc[k][rank]) return fail("exchange counts disagree");
      if (!n) continue;
      const char* s = static_cast<const char*>(hub->src[k]) + hub->sd[k][rank] * elem;
      if (hipMemcpyAsync(static_cast<char*>(recv) + rdispls[k] * elem, s, n * elem, hipMemcpyDeviceToDevice, st) !=
          hipSuccess)
        return fail("exchange copy");
    }
    if (hipStreamSynchronize(st) != hipSuccess) return fail("stream sync after exchange");
    if (!hub->barrier()) return fail("exchange aborted by another shard");
    return true;
  }
  // small arrays make a host round trip: every shard's values are gathered, combined, written back
  template <class T, class F>
  bool host_collective(const T* in, T* out, size_t count, bool gather, hipStream_t st, F comb) {
    std::vector<T> mine(count);
    if (hipMemcpyAsync(mine.data(), in, sizeof(T) * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail("collective copy");
    hub->vals[rank].assign(mine.begin(), mine.end());
    if (!hub->barrier()) return fail("collective aborted by another shard");
    std::vector<T> res(gather ? count * world : count);
    for (size_t q = 0; q < count; ++q) {
      if (gather) {
        for (int k = 0; k < world; ++k) res[k * count + q] = (T)hub->vals[k][q];
      } else {
        T a = (T)hub->vals[0][q];
        for (int k = 1; k < world; ++k) a = comb(a, (T)hub->vals[k][q]);
        res[q] = a;
      }
    }
    if (!hub->barrier()) return fail("collective aborted by another shard");
    if (hipMemcpyAsync(out, res.data(), sizeof(T) * res.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail("collective copy back");
    return true;
  }
  bool allgather_u32(const uint32_t* send, uint32_t* recv, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(send, recv, count, true, st, [](uint32_t a, uint32_t) { return a; });
  }
  bool allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(buf, buf, count, false, st, [](uint32_t a, uint32_t b) { return a + b; });
  }
  bool allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(buf, buf, count, false, st, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
  }
  bool allreduce_sum_u64(unsigned long long* buf, size_t count, hipStream_t st) override {
    return host_collective<unsigned long long>(buf, buf, count, false, st,
                                               [](unsigned long long a, unsigned long long b) { return a + b; });
  }
  std::string error() const override { return "local exchange: " + err; }
};

// ---- ranks in separate processes on ONE device (test transport) -------------------------------
// RCCL refuses two ranks on one GPU, so kb_sim_create_rank's multi-process path could not be exercised on
// a one-GPU box.  IpcXfer carries the same exchange between processes that share a device: each rank
// exports one device window (hipIpcGetMemHandle; dmabuf IPC) through a POSIX shared-memory segment that
// also holds the rendezvous (a process-shared barrier), every rank's counts and displacements, and the
// values of the small collectives.  An all-to-all-v copies the rank's send data into its own window,
// meets the others, pulls its receive blocks from their windows (device-to-device copies on its own
// stream) and meets them again before any window is reused.  The product transport stays RcclXfer.
constexpr uint32_t IPC_VALS = 256;                        // values per rank of a small collective
constexpr char IPC_MAGIC[8] = {'K', 'B', 'I', 'P', 'C', '1', 0, 0};   // kb_ipc_unique_id's prefix
struct IpcShared {
  std::atomic<uint32_t> arrived, aborted, opened;
  std::atomic<uint64_t> gen;
  hipIpcMemHandle_t handle[XMAX];
  uint64_t wbytes[XMAX];
  uint64_t sc[XMAX][XMAX], sd[XMAX][XMAX];               // rank k's send counts / displacements (elements)
  unsigned long long vals[XMAX][IPC_VALS];
};
struct IpcXfer : Xfer {
  IpcShared* sh = nullptr;
  size_t shsz = sizeof(IpcShared);
  char* win = nullptr;                                   // this rank's window
  size_t wbytes = 0;
  std::vector<char*> peer;                               // the other ranks' windows, mapped here
  std::string err, name;
  bool unlinked = false;
  // rank 0 created the segment's name: every failure path removes it (no /dev/shm leftovers from failed runs)
  void unlink_name() { if (rank == 0 && !name.empty() && !unlinked) { shm_unlink(name.c_str()); unlinked = true; } }
  bool fail(const std::string& what) { err = what; if (sh) sh->aborted.store(1); unlink_name(); return false; }
  bool barrier() {
    const uint64_t g = sh->gen.load(std::memory_order_acquire);
    if (sh->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)world) {
      sh->arrived.store(0, std::memory_order_relaxed);
      sh->gen.fetch_add(1, std::memory_order_release);
      return !sh->aborted.load();
    }
    for (uint64_t spin = 0; sh->gen.load(std::memory_order_acquire) == g; ++spin) {
      if (sh->aborted.load()) return false;
      if (spin > 1000) usleep(spin > 100000 ? 1000 : 20);
      if (spin > 100000 + 120000) { err = "IPC barrier timed out (a rank is gone)"; sh->aborted.store(1); return false; }
    }
    return !sh->aborted.load();
  }
  // uid = IPC_MAGIC + the segment's name (kb_ipc_unique_id)
  bool init(int r, int w, const void* uid, size_t window_bytes) {
    rank = r; world = w; wbytes = window_bytes;
    name.assign(static_cast<const char*>(uid) + sizeof IPC_MAGIC);
    const int fd = shm_open(name.c_str(), O_RDWR | (r == 0 ? O_CREAT : 0), 0600);
    int fd2 = fd;
    for (int t = 0; fd2 < 0 && r != 0 && t < 20000; ++t) { usleep(1000); fd2 = shm_open(name.c_str(), O_RDWR, 0600); }
    if (fd2 < 0) { err = "shm_open " + name; return false; }
    if (r == 0 && ftruncate(fd2, (off_t)shsz) != 0) { close(fd2); return fail("ftruncate"); }
    struct stat stt;
    for (int t = 0; t < 20000; ++t) { if (fstat(fd2, &stt) == 0 && (size_t)stt.st_size >= shsz) break; usleep(1000); }
    void* p = mmap(nullptr, shsz, PROT_READ | PROT_WRITE, MAP_SHARED, fd2, 0);
    close(fd2);
    if (p == MAP_FAILED) return fail("mmap");
    sh = static_cast<IpcShared*>(p);                      // zero-filled by ftruncate: counters start at 0
    if (hipMalloc((void**)&win, wbytes) != hipSuccess) return fail("window allocation");
    if (hipIpcGetMemHandle(&sh->handle[r], win) != hipSuccess) return fail("hipIpcGetMemHandle");
    sh->wbytes[r] = wbytes;
    sh->opened.fetch_add(1);
    for (int t = 0; sh->opened.load() < (uint32_t)w; ++t) {      // every rank attached and exported its window
      if (t > 120000) return fail("IPC: not every rank attached");
      usleep(1000);
    }
    peer.assign(w, nullptr);
    for (int k = 0; k < w; ++k) {
      if (k == r) { peer[k] = win; continue; }
      void* q = nullptr;
      if (hipIpcOpenMemHandle(&q, sh->handle[k], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return fail("hipIpcOpenMemHandle");
      peer[k] = static_cast<char*>(q);
    }
    if (!barrier()) return fail("IPC attach barrier");
    unlink_name();                                        // every rank has it mapped: no name left behind
    return true;
  }
  ~IpcXfer() override {
    for (int k = 0; k < (int)peer.size(); ++k) if (k != rank && peer[k]) (void)hipIpcCloseMemHandle(peer[k]);
    if (win) (void)hipFree(win);
    if (sh) munmap(sh, shsz);
  }
  void abort() override { if (sh) sh->aborted.store(1); }
  bool alltoallv(const void* send, const size_t* scounts, const size_t* sdispls, void* recv, const size_t* rcounts,
                 const size_t* rdispls, size_t elem, hipStream_t st) override {
    for (int k = 0; k < world; ++k) {
      if ((sdispls[k] + scounts[k]) * elem > wbytes) return fail("IPC window too small (KB_IPC_WINDOW_MB)");
      sh->sc[rank][k] = scounts[k]; sh->sd[rank][k] = sdispls[k];
      if (scounts[k] && hipMemcpyAsync(win + sdispls[k] * elem, static_cast<const char*>(send) + sdispls[k] * elem,
                                       scounts[k] * elem, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail("IPC window copy");
    }
    if (hipStreamSynchronize(st) != hipSuccess) return fail("stream sync before exchange");
    if (!barrier()) return fail(err.empty() ? "exchange aborted by another rank" : err);
    for (int k = 0; k < world; ++k) {
      const size_t n = rcounts[k];
      if (n != sh->sc[k][rank]) return fail("exchange counts disagree");
      if (n && hipMemcpyAsync(static_cast<char*>(recv) + rdispls[k] * elem, peer[k] + sh->sd[k][rank] * elem, n * elem,
                              hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail("IPC exchange copy");
    }
    if (hipStreamSynchronize(st) != hipSuccess) return fail("stream sync after exchange");
    if (!barrier()) return fail(err.empty() ? "exchange aborted by another rank" : err);
    return true;
  }
  template <class T, class F>
  bool host_collective(const T* in, T* out, size_t count, bool gather, hipStream_t st, F comb) {
    if (count > IPC_VALS) return fail("IPC collective too large");
    std::vector<T> mine(count);
    if (hipMemcpyAsync(mine.data(), in, sizeof(T) * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail("collective copy");
    for (size_t q = 0; q < count; ++q) sh->vals[rank][q] = (unsigned long long)mine[q];
    if (!barrier()) return fail("collective aborted by another rank");
    std::vector<T> res(gather ? count * world : count);
    for (size_t q = 0; q < count; ++q) {
      if (gather) {
        for (int k = 0; k < world; ++k) res[k * count + q] = (T)sh->vals[k][q];
      } else {
        T a = (T)sh->vals[0][q];
        for (int k = 1; k < world; ++k) a = comb(a, (T)sh->vals[k][q]);
        res[q] = a;
      }
    }
    if (!barrier()) return fail("collective aborted by another rank");
    if (hipMemcpyAsync(out, res.data(), sizeof(T) * res.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail("collective copy back");
    return true;
  }
  bool allgather_u32(const uint32_t* send, uint32_t* recv, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(send, recv, count, true, st, [](uint32_t a, uint32_t) { return a; });
  }
  bool allreduce_sum_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(buf, buf, count, false, st, [](uint32_t a, uint32_t b) { return a + b; });
  }
  bool allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t st) override {
    return host_collective<uint32_t>(buf, buf, count, false, st, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
  }
  bool allreduce_sum_u64(unsigned long long* buf, size_t count, hipStream_t st) override {
    return host_collective<unsigned long long>(buf, buf, count, false, st,
                                               [](unsigned long long a, unsigned long long b) { return a + b; });
  }
  std::string error() const override { return "IPC exchange: " + err; }
};

}  // namespace kb
