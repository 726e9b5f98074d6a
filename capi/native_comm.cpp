// Transports of multi-process native contexts (see native_comm.h): RCCL loaded at run time (dlopen, so
// a program that never builds a multi-process context does not load it, and the library never clashes
// with the copy a Python process may already hold) and the node-local file transport.
#include "native_comm.h"

#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <thread>
#include <type_traits>

#include "native_internal.h"

namespace {

double timeout_s() {
  const char* v = std::getenv("DPLASMA_NATIVE_TIMEOUT");
  return v && *v ? std::atof(v) : 600.0;
}

bool write_file(const std::string& dir, const std::string& name, const void* data, size_t bytes) {
  const std::string tmp = dir + "/.tmp." + name, fin = dir + "/" + name;
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return false;
  const bool ok = (bytes == 0 || std::fwrite(data, 1, bytes, f) == bytes) && std::fclose(f) == 0;
  return ok && std::rename(tmp.c_str(), fin.c_str()) == 0;   // readers only ever see complete files
}

// wait for dir/name (written by write_file), read exactly bytes, optionally remove it
bool read_file(const std::string& dir, const std::string& name, void* data, size_t bytes, bool remove) {
  const std::string fin = dir + "/" + name;
  const auto t0 = std::chrono::steady_clock::now();
  int us = 5;
  FILE* f = nullptr;
  while (!(f = std::fopen(fin.c_str(), "rb"))) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s()) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = std::min(us * 2, 2000);
  }
  const bool ok = bytes == 0 || std::fread(data, 1, bytes, f) == bytes;
  std::fclose(f);
  if (remove) std::remove(fin.c_str());
  return ok;
}

// ------------------------------------------------------------------------------------------ files
bool debug() {
  static const int v = [] { const char* e = std::getenv("DPLASMA_NATIVE_DEBUG"); return e && *e == '1' ? 1 : 0; }();
  return v == 1;
}

class FileComm final : public NatComm {
 public:
  std::string dir, token;   // token: this job's session (see nat_comm_create), prefix of every message
  std::vector<long long> sseq, rseq;   // per-peer message counters (pairs match in issue order)
  std::vector<char> stage;

  const char* name() const override { return "file"; }

  bool send_host(int peer, const void* p, size_t bytes) {
    const std::string n = "m." + token + "." + std::to_string(rank) + "." + std::to_string(peer) + "." +
                          std::to_string(sseq[peer]++);
    return write_file(dir, n, p, bytes);
  }
  bool recv_host(int peer, void* p, size_t bytes) {
    const std::string n = "m." + token + "." + std::to_string(peer) + "." + std::to_string(rank) + "." +
                          std::to_string(rseq[peer]++);
    return read_file(dir, n, p, bytes, true);
  }

  int exchange(const std::vector<NatMsg>& sends, const std::vector<NatMsg>& recvs, hipStream_t st) override {
    if (sends.empty() && recvs.empty()) return 0;
    if (debug()) {
      std::fprintf(stderr, "[native rank %d] exchange: %zu sends (", rank, sends.size());
      for (const NatMsg& m : sends) std::fprintf(stderr, " %d", m.peer);
      std::fprintf(stderr, " ), %zu recvs (", recvs.size());
      for (const NatMsg& m : recvs) std::fprintf(stderr, " %d", m.peer);
      std::fprintf(stderr, " )\n");
    }
    if (hipStreamSynchronize(st) != hipSuccess) return -1;   // the producers of the sends are done
    for (const NatMsg& m : sends) {
      stage.resize(m.bytes);
      if (hipMemcpy(stage.data(), m.buf, m.bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
      if (!send_host(m.peer, stage.data(), m.bytes)) return -2;
    }
    for (const NatMsg& m : recvs) {   // sends never wait for receivers: no exchange can deadlock
      stage.resize(m.bytes);
      if (!recv_host(m.peer, stage.data(), m.bytes)) return -3;
      if (hipMemcpy(m.buf, stage.data(), m.bytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
    }
    return 0;
  }

  int allreduce(double* v, int n, bool max) override {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const size_t b = sizeof(double) * n;
    if (rank == 0) {
      std::vector<double> o(n);
      for (int r = 1; r < world; ++r) {
        if (!recv_host(r, o.data(), b)) return -3;
        for (int i = 0; i < n; ++i) v[i] = max ? std::max(v[i], o[i]) : v[i] + o[i];
      }
      for (int r = 1; r < world; ++r)
        if (!send_host(r, v, b)) return -2;
      return 0;
    }
    return send_host(0, v, b) && recv_host(0, v, b) ? 0 : -3;
  }
};

// ------------------------------------------------------------------------------------------- RCCL
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*errorString)(ncclResult_t) = nullptr;

  bool load(std::string& err) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) { err = "librccl.so.1 not found"; return false; }
    bool ok = true;
    auto sym = [&](auto& fp, const char* n) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, n));
      ok = ok && fp;
    };
    sym(getUniqueId, "ncclGetUniqueId");
    sym(commInitRank, "ncclCommInitRank");
    sym(commDestroy, "ncclCommDestroy");
    sym(send, "ncclSend");
    sym(recv, "ncclRecv");
    sym(groupStart, "ncclGroupStart");
    sym(groupEnd, "ncclGroupEnd");
    sym(allReduce, "ncclAllReduce");
    sym(errorString, "ncclGetErrorString");
    if (!ok) err = "librccl.so.1 lacks a symbol";
    return ok;
  }
};

class RcclComm final : public NatComm {
 public:
  Rccl r;
  ncclComm_t comm = nullptr;
  hipStream_t st = nullptr;   // host all-reduces
  double* scratch = nullptr;
  int scratch_n = 0;

  const char* name() const override { return "rccl"; }
  ~RcclComm() override {
    if (comm) r.commDestroy(comm);
    if (scratch) (void)hipFree(scratch);
    if (st) (void)hipStreamDestroy(st);
  }

  int exchange(const std::vector<NatMsg>& sends, const std::vector<NatMsg>& recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return 0;
    if (debug())
      std::fprintf(stderr, "[native rank %d] rccl exchange: %zu sends, %zu recvs\n", rank, sends.size(), recvs.size());
    if (r.groupStart() != ncclSuccess) return -1;
    ncclResult_t e = ncclSuccess;
    for (const NatMsg& m : sends)
      if (e == ncclSuccess) e = r.send(m.buf, m.bytes, ncclUint8, m.peer, comm, s);
    for (const NatMsg& m : recvs)
      if (e == ncclSuccess) e = r.recv(m.buf, m.bytes, ncclUint8, m.peer, comm, s);
    const ncclResult_t g = r.groupEnd();
    return e == ncclSuccess && g == ncclSuccess ? 0 : -1;
  }

  int allreduce(double* v, int n, bool max) override {
    if (n > scratch_n) {
      if (scratch) (void)hipFree(scratch);
      scratch = nullptr;
      if (hipMalloc(&scratch, sizeof(double) * n) != hipSuccess) return -1;
      scratch_n = n;
    }
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(scratch, v, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess)
      return -1;
    if (r.allReduce(scratch, scratch, n, ncclFloat64, max ? ncclMax : ncclSum, comm, st) != ncclSuccess) return -1;
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(v, scratch, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    return 0;
  }
};

}  // namespace

// ------------------------------------------------------------------------------------------ session
// Rendezvous in a node-local directory, safe against files an earlier (crashed) job left there:
//   rank 0 removes every stale rendezvous file, draws a random session token T and publishes it
//   ("session"); every other rank draws a random nonce, reads T and answers "hello.T.r" = {nonce, its
//   transport preference}; rank 0, once it has every hello, decides the transport for everyone (RCCL
//   only if every rank sees enough GPUs and DPLASMA_NATIVE_TRANSPORT at rank 0 does not say "file")
//   and publishes "go.T" = {transport, every rank's nonce, the RCCL unique id}.  A rank accepts a go
//   file only if it carries its own nonce, and re-answers if the session token changes while it
//   waits -- a stale session, hello or go file is never taken for this job's.  Message files are
//   named m.T.src.dst.seq.
namespace {

unsigned long long rnd64() {
  unsigned long long v = 0;
  if (FILE* f = std::fopen("/dev/urandom", "rb")) {
    if (std::fread(&v, sizeof v, 1, f) != 1) v = 0;
    std::fclose(f);
  }
  if (v == 0)
    v = (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count() ^
        ((unsigned long long)getpid() << 32);
  return v;
}

std::string hex(unsigned long long v) {
  char b[17];
  std::snprintf(b, sizeof b, "%016llx", v);
  return b;
}

struct Session {
  unsigned long long token;
  int world;
};
struct Hello {
  unsigned long long nonce;
  int pref_rccl;
  int pad;
};
struct GoHead {
  int rccl;
  int world;
  ncclUniqueId id;
};

bool try_read(const std::string& path, void* data, size_t bytes) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  const bool ok = std::fread(data, 1, bytes, f) == bytes;
  std::fclose(f);
  return ok;
}

// Removes rendezvous files older than the transport timeout only: every hello / go / message file is named
// by its session token, so a younger file (another job sharing the directory, or a peer of a restarted job
// still draining) can never be taken for this session's and is left alone; "session" itself is rewritten
// atomically, which a running job no longer reads.
void remove_stale(const std::string& dir) {
  const double max_age = timeout_s();
  const time_t now = time(nullptr);
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      const std::string n = e->d_name;
      if (!(n == "session" || n.rfind("hello.", 0) == 0 || n.rfind("go.", 0) == 0 || n.rfind("m.", 0) == 0 ||
            n.rfind(".tmp.", 0) == 0))
        continue;
      struct stat st {};
      const std::string path = dir + "/" + n;
      if (stat(path.c_str(), &st) == 0 && difftime(now, st.st_mtime) > max_age) std::remove(path.c_str());
    }
    closedir(d);
  }
}

// establishes the session; returns false (err set) on timeout
bool rendezvous(const std::string& dir, int rank, int world, bool pref_rccl, const Rccl* rccl, std::string& token,
                bool& use_rccl, ncclUniqueId& id, std::string& err) {
  const auto t0 = std::chrono::steady_clock::now();
  auto expired = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s(); };
  if (rank == 0) {
    remove_stale(dir);
    const Session ss{rnd64(), world};
    token = hex(ss.token);
    if (!write_file(dir, "session", &ss, sizeof ss)) { err = "cannot write the session file in " + dir; return false; }
    std::vector<unsigned long long> nonces(world, 0);
    bool all_rccl = pref_rccl;
    for (int r = 1; r < world; ++r) {
      Hello h{};
      if (!read_file(dir, "hello." + token + "." + std::to_string(r), &h, sizeof h, true)) {
        err = "native rendezvous: rank " + std::to_string(r) + " did not answer in " + dir;
        return false;
      }
      nonces[r] = h.nonce;
      all_rccl = all_rccl && h.pref_rccl;
    }
    const char* tv = std::getenv("DPLASMA_NATIVE_TRANSPORT");
    use_rccl = tv && *tv ? std::string(tv) == "rccl" : all_rccl;
    GoHead gh{};
    gh.rccl = use_rccl ? 1 : 0;
    gh.world = world;
    if (use_rccl && (!rccl || rccl->getUniqueId(&gh.id) != ncclSuccess)) { err = "RCCL unique id"; return false; }
    id = gh.id;
    std::vector<char> buf(sizeof gh + sizeof(unsigned long long) * world);
    std::memcpy(buf.data(), &gh, sizeof gh);
    std::memcpy(buf.data() + sizeof gh, nonces.data(), sizeof(unsigned long long) * world);
    if (!write_file(dir, "go." + token, buf.data(), buf.size())) { err = "cannot write the go file"; return false; }
    return true;
  }
  const unsigned long long nonce = rnd64();
  std::string cur_tok;
  int us = 50;
  while (!expired()) {
    Session ss{};
    if (!try_read(dir + "/session", &ss, sizeof ss) || ss.world != world) {
      std::this_thread::sleep_for(std::chrono::microseconds(us));
      us = std::min(2 * us, 5000);
      continue;
    }
    const std::string tok = hex(ss.token);
    if (tok != cur_tok) {   // (re)answer this session
      const Hello h{nonce, pref_rccl ? 1 : 0, 0};
      if (!write_file(dir, "hello." + tok + "." + std::to_string(rank), &h, sizeof h)) { err = "cannot write hello"; return false; }
      cur_tok = tok;
    }
    std::vector<char> buf(sizeof(GoHead) + sizeof(unsigned long long) * world);
    if (try_read(dir + "/go." + tok, buf.data(), buf.size())) {
      GoHead gh;
      std::memcpy(&gh, buf.data(), sizeof gh);
      unsigned long long mine = 0;
      std::memcpy(&mine, buf.data() + sizeof gh + sizeof(unsigned long long) * rank, sizeof mine);
      if (gh.world == world && mine == nonce) {
        token = tok;
        use_rccl = gh.rccl != 0;
        id = gh.id;
        return true;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = std::min(2 * us, 5000);
  }
  err = "native rendezvous timed out in " + dir;
  return false;
}

}  // namespace

// Rank replay on one GPU (DPLASMA_NATIVE_TRANSPORT=replay; tools/replay_native.py): this process is rank
// `rank` of a `world`-rank grid with no peers.  An exchange moves no data: it is one busy-wait kernel on the
// communication stream lasting lat + (the busiest peer link's bytes) / bw -- the timing model of
// tools/replay_potrf.py's ReplayBackend without producer proxies (DPLASMA_REPLAY_BW GB/s per link,
// DPLASMA_REPLAY_LAT us per exchange, DPLASMA_REPLAY_WG workgroups).  Host all-reduces return the local value.
extern "C" int dpl_delay(double us, int nwg, hipStream_t st);
class ReplayComm final : public NatComm {
 public:
  double bw = 50e3, lat = 15.0;   // bytes per us, us
  int nwg = 4;
  long long batches = 0;
  double total_us = 0;
  const char* name() const override { return "replay"; }
  int exchange(const std::vector<NatMsg>& sends, const std::vector<NatMsg>& recvs, hipStream_t s) override {
    if (sends.empty() && recvs.empty()) return 0;
    std::vector<double> per(world, 0.0);
    for (const NatMsg& m : sends) per[m.peer] += (double)m.bytes;
    for (const NatMsg& m : recvs) per[m.peer] += (double)m.bytes;
    double mx = 0;
    for (double v : per) mx = std::max(mx, v);
    const double us = lat + mx / bw;
    ++batches;
    total_us += us;
    return dpl_delay(us, nwg, s);
  }
  int allreduce(double*, int, bool) override { return 0; }
  ~ReplayComm() override {
    if (std::getenv("DPLASMA_REPLAY_STATS"))
      std::fprintf(stderr, "[replay rank %d] %lld exchanges, %.1f us modelled\n", rank, batches, total_us);
  }
};

NatComm* nat_comm_create(int rank, int world, int device, const char* rdv_dir, std::string& err) {
  {
    const char* tv = std::getenv("DPLASMA_NATIVE_TRANSPORT");
    if (tv && std::string(tv) == "replay") {
      auto* c = new ReplayComm;
      c->rank = rank;
      c->world = world;
      const char* v;
      if ((v = std::getenv("DPLASMA_REPLAY_BW")) && *v) c->bw = std::atof(v) * 1e3;
      if ((v = std::getenv("DPLASMA_REPLAY_LAT")) && *v) c->lat = std::atof(v);
      if ((v = std::getenv("DPLASMA_REPLAY_WG")) && *v) c->nwg = std::max(1, std::atoi(v));
      (void)device;
      (void)rdv_dir;
      return c;
    }
  }
  const char* env_dir = std::getenv("DPLASMA_NATIVE_RDV");
  const std::string dir = rdv_dir && *rdv_dir ? rdv_dir : env_dir ? env_dir : "";
  if (dir.empty()) { err = "no rendezvous directory (argument or DPLASMA_NATIVE_RDV)"; return nullptr; }
  (void)mkdir(dir.c_str(), 0700);
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  const char* tv = std::getenv("DPLASMA_NATIVE_TRANSPORT");
  const std::string want = tv && *tv ? tv : "";
  if (!want.empty() && want != "rccl" && want != "file") { err = "DPLASMA_NATIVE_TRANSPORT must be rccl, file or replay"; return nullptr; }
  // this rank's preference; rank 0 decides for everyone (a per-rank choice could split the job)
  const bool pref_rccl = want.empty() ? ndev >= world : want == "rccl";
  Rccl rccl;
  std::string rerr;
  const bool have_rccl = rccl.load(rerr);
  std::string token;
  bool use_rccl = false;
  ncclUniqueId id{};
  if (!rendezvous(dir, rank, world, pref_rccl && have_rccl, have_rccl ? &rccl : nullptr, token, use_rccl, id, err))
    return nullptr;
  if (!use_rccl) {
    auto* c = new FileComm;
    c->rank = rank;
    c->world = world;
    c->dir = dir;
    c->token = token;
    c->session_token = token;
    c->sseq.assign(world, 0);
    c->rseq.assign(world, 0);
    double x = 0.0;   // every rank present before the first exchange
    if (c->allreduce(&x, 1, false) != 0) { err = "file transport: rendezvous timed out in " + dir; delete c; return nullptr; }
    c->session_dir = dir;
    return c;
  }
  if (!have_rccl) { err = "rank 0 chose RCCL but " + rerr; return nullptr; }
  auto* c = new RcclComm;
  c->rank = rank;
  c->world = world;
  c->r = rccl;
  (void)hipSetDevice(device);
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, hi) != hipSuccess ||
      c->r.commInitRank(&c->comm, world, id, rank) != ncclSuccess) {
    err = "ncclCommInitRank failed";
    delete c;
    return nullptr;
  }
  double x = 0.0;
  if (c->allreduce(&x, 1, false) != 0) { err = "RCCL all-reduce failed"; delete c; return nullptr; }
  c->session_dir = dir;
  c->session_token = token;
  return c;
}

void nat_comm_destroy(NatComm* c) {
  double x = 0.0;   // nobody leaves while a peer may still read its messages
  (void)c->allreduce(&x, 1, false);
  if (c->rank == 0 && !c->session_dir.empty()) {   // the session's files: nobody reads them any more
    std::remove((c->session_dir + "/session").c_str());
    if (!c->session_token.empty()) std::remove((c->session_dir + "/go." + c->session_token).c_str());
  }
  delete c;
}

int nat_comm_reduce_info(NatComm* c, int& info) {
  double v[2] = {info > 0 ? -(double)info : -1e300, info < 0 ? 1.0 : 0.0};
  if (c->allreduce(v, 2, true) != 0) return -1;
  info = v[1] > 0 ? -1 : v[0] > -1e300 ? (int)-v[0] : 0;
  return 0;
}
