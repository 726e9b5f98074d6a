// Tile transport of a multi-process native context (native_dist.cpp).
//
// The reference moves tiles between MPI ranks through PaRSEC's remote dependencies (the JDF edges
// of src/zpotrf_L.jdf:140-188, src/zgemm_NN_summa.jdf); here a step's every send and receive is ONE
// grouped point-to-point exchange issued on the context's communication stream:
//   * RCCL (one GPU per rank, xGMI): ncclSend / ncclRecv inside ncclGroupStart / End, stream ordered
//     -- no host synchronisation, the exchange overlaps the update stream;
//   * files (ranks sharing one GPU, where RCCL refuses to build a communicator; rehearsals and tests):
//     the exchange drains its stream, stages each message through host memory into a node-local file
//     of the rendezvous directory, and blocks until its receives have arrived.
// Messages between one pair of ranks match in issue order (both transports), so the builders only
// have to enumerate every exchange's messages in the same order on both sides.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>
#include <vector>

struct NatMsg {
  int peer;
  void* buf;       // device memory of the context's GPU
  size_t bytes;
};

class NatComm {
 public:
  int rank = 0, world = 1;
  std::string session_dir, session_token;   // rendezvous session (native_comm.cpp), cleaned up by rank 0
  virtual ~NatComm() = default;
  virtual const char* name() const = 0;
  // every send and receive of one step, issued on stream st after the work already queued there
  virtual int exchange(const std::vector<NatMsg>& sends, const std::vector<NatMsg>& recvs, hipStream_t st) = 0;
  // host all-reduce of n doubles (sum, or max), after the device work queued so far
  virtual int allreduce(double* v, int n, bool max) = 0;
};
