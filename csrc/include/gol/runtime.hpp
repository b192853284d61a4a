// gol-mi355x: process runtime — launch-mode detection, bootstrap, device selection and the
// reference-compatible CLI driver.
//
// Launch modes (first match wins):
//   GOL_NRANKS=P (P > 1)          P ranks as threads of this process (one GPU each, rank % ngpu)
//   mpirun / mpiexec (PMI env)    MPI bootstrap (when built with MPI)       — reference contract
//   RANK/WORLD_SIZE (torchrun)    TCP rendezvous on MASTER_ADDR:MASTER_PORT
//   otherwise                     single rank
// On the HIP backend with P > 1 the halo data plane is RCCL over the chosen control plane.
#pragma once

#include <memory>
#include <string>

#include "gol/config.hpp"
#include "gol/engine.hpp"
#include "gol/transport.hpp"

namespace gol {

struct LaunchInfo {
    std::string mode = "single";  // single | threads | mpi | tcp
    int rank = 0, size = 1, local_rank = 0;
};

// Detect the launch mode from the environment (does not create anything).
LaunchInfo detect_launch(const Options& o);

// Control-plane transport for a process launch (single / mpi / tcp).
std::shared_ptr<Transport> make_control_transport(const LaunchInfo& li, int* argc, char*** argv);

// Pick the backend ("auto" -> hip when a device exists).  For hip, selects device local_rank % n
// and throws ContractError with the reference's messages (gol-with-cuda.cu:290-300) on failure.
std::string select_backend(const Options& o, int rank, int local_rank);

// Wrap a control plane with RCCL when the backend is hip, P > 1 and every rank has its own GPU
// (`device` must be current).  Ranks sharing a GPU, or GOL_TRANSPORT=host, stage halos through host
// memory over the control plane instead.
std::shared_ptr<Transport> make_data_transport(std::shared_ptr<Transport> control, const std::string& backend,
                                               const Options& o, int device);

EngineConfig engine_config(const Options& o, const std::string& backend, int device);

// CLI threadsPerBlock as a hint: the LDS tile kernel's workgroup size (T/64 waves).  Values that
// are not a multiple of 64 in 64..1024 warn on stderr (when `report`) and keep the default.
void apply_threads_hint(EngineConfig& c, unsigned threads, bool report);

// The `gol` program: ./gol <pattern> <worldSize> <iterations> <threadsPerBlock> <output_on_off>.
// Returns the process exit status.
int run_cli(int argc, char** argv);

// Write the per-rank dump files for the current engine state (collective).  `fp` is this rank's
// open file (reference opens it before init, gol-main.c:64-73).
void write_dumps(Engine& eng, FILE* fp);

// Checkpoint I/O (GOL_CHECKPOINT_EVERY / GOL_RESTART): one binary snapshot per rank.
void save_checkpoint(Engine& eng, const std::string& prefix, u64 seed);
u64 load_checkpoint(Engine& eng, const std::string& prefix);  // returns the snapshot generation

}  // namespace gol
