// Transports of multi-process native contexts (see native_comm.h): RCCL loaded at run time (dlopen, so
// a program that never builds a multi-process context does not load it, and the library never clashes
// with the copy a Python process may already hold) and the node-local file transport.
#include "native_comm.h"

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
  std::string dir;
  std::vector<long long> sseq, rseq;   // per-peer message counters (pairs match in issue order)
  std::vector<char> stage;

  const char* name() const override { return "file"; }

  bool send_host(int peer, const void* p, size_t bytes) {
    const std::string n = "m." + std::to_string(rank) + "." + std::to_string(peer) + "." + std::to_string(sseq[peer]++);
    return write_file(dir, n, p, bytes);
  }
  bool recv_host(int peer, void* p, size_t bytes) {
    const std::string n = "m." + std::to_string(peer) + "." + std::to_string(rank) + "." + std::to_string(rseq[peer]++);
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

NatComm* nat_comm_create(int rank, int world, int device, const char* rdv_dir, std::string& err) {
  const char* env_dir = std::getenv("DPLASMA_NATIVE_RDV");
  const std::string dir = rdv_dir && *rdv_dir ? rdv_dir : env_dir ? env_dir : "";
  if (dir.empty()) { err = "no rendezvous directory (argument or DPLASMA_NATIVE_RDV)"; return nullptr; }
  (void)mkdir(dir.c_str(), 0700);
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  const char* tv = std::getenv("DPLASMA_NATIVE_TRANSPORT");
  const std::string t = tv && *tv ? tv : (ndev >= world ? "rccl" : "file");
  if (t == "file") {
    auto* c = new FileComm;
    c->rank = rank;
    c->world = world;
    c->dir = dir;
    c->sseq.assign(world, 0);
    c->rseq.assign(world, 0);
    double x = 0.0;   // every rank present before the first exchange
    if (c->allreduce(&x, 1, false) != 0) { err = "file transport: rendezvous timed out in " + dir; delete c; return nullptr; }
    return c;
  }
  if (t != "rccl") { err = "DPLASMA_NATIVE_TRANSPORT must be rccl or file"; return nullptr; }
  auto* c = new RcclComm;
  c->rank = rank;
  c->world = world;
  if (!c->r.load(err)) { delete c; return nullptr; }
  ncclUniqueId id;
  if (rank == 0) {
    if (c->r.getUniqueId(&id) != ncclSuccess || !write_file(dir, "ncclid", &id, sizeof id)) {
      err = "RCCL unique id";
      delete c;
      return nullptr;
    }
  } else if (!read_file(dir, "ncclid", &id, sizeof id, false)) {
    err = "RCCL rendezvous timed out in " + dir;
    delete c;
    return nullptr;
  }
  (void)hipSetDevice(device);
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, hi) != hipSuccess ||
      c->r.commInitRank(&c->comm, world, id, rank) != ncclSuccess) {
    err = "ncclCommInitRank failed";
    delete c;
    return nullptr;
  }
  double x = 0.0;   // everyone has read the id: rank 0 removes it
  if (c->allreduce(&x, 1, false) != 0) { err = "RCCL all-reduce failed"; delete c; return nullptr; }
  if (rank == 0) std::remove((dir + "/ncclid").c_str());
  return c;
}

void nat_comm_destroy(NatComm* c) {
  double x = 0.0;   // nobody leaves while a peer may still read its messages
  (void)c->allreduce(&x, 1, false);
  delete c;
}

int nat_comm_reduce_info(NatComm* c, int& info) {
  double v[2] = {info > 0 ? -(double)info : -1e300, info < 0 ? 1.0 : 0.0};
  if (c->allreduce(v, 2, true) != 0) return -1;
  info = v[1] > 0 ? -1 : v[0] > -1e300 ? (int)-v[0] : 0;
  return 0;
}
