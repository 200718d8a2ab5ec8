// mdfx process bootstrap for the native CLIs: rank discovery from the launcher environment and a
// small TCP rendezvous (no MPI library needed).
//
// Reference parity: MPI_Init / MPI_Comm_rank / MPI_Comm_size (MDF_kernel.cu:128-131) plus the
// stdin config every rank read for itself (D14). Here `mpirun -np N ./mdf` (MPICH hydra sets
// PMI_RANK/PMI_SIZE), Open MPI (OMPI_COMM_WORLD_*) and torchrun (RANK/WORLD_SIZE) all work: rank 0
// reads the dialogue and broadcasts it, and the RCCL unique id travels the same way.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "mdfx/runtime.hpp"

namespace mdfx {

struct ProcEnv {
  int rank = 0;
  int world = 1;
  int local_rank = 0;
  bool launched = false;       // started by a multi-process launcher
  std::string addr = "127.0.0.1";
  int port = 29533;
};
ProcEnv detect_proc_env();

// Star rendezvous through rank 0 over TCP. All collectives are blocking and must be called by
// every rank in the same order.
class Rendezvous {
 public:
  Rendezvous(const ProcEnv& env, double timeout_s = 120.0);
  ~Rendezvous();
  int rank() const { return env_.rank; }
  int world() const { return env_.world; }
  std::string bcast(const std::string& root_data);
  std::vector<std::string> allgather(const std::string& mine);
  double allreduce_max(double v);
  double allreduce_sum(double v);
  void barrier();

 private:
  ProcEnv env_;
  int listen_fd_ = -1;
  std::vector<int> peers_;  // root: fd per rank (index = rank); others: [fd to root]
};

// Host-memory halo transport between processes over TCP (CPU backend, one slab per process):
// each rank keeps one full-duplex socket to each slab neighbour.
std::unique_ptr<Transport> make_tcp_transport(Rendezvous& rv);

}  // namespace mdfx
