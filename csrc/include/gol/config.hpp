// gol-mi355x: command line + environment configuration.
//
// The CLI is byte-compatible with the reference (gol-main.c:33-53): exactly 5 positional arguments,
// each parsed with atoi into the reference's types (threadsPerBlock is an unsigned short, so it
// truncates mod 65536), and a wrong argument count prints the reference usage line and exits with
// status 255 before any communicator is created.  Every extension is an environment variable
// (GOL_*), so command lines written for the reference keep working unchanged.
#pragma once

#include <string>

#include "gol/common.hpp"

namespace gol {

struct CliArgs {
    unsigned pattern = 0;
    unsigned world_size = 0;
    unsigned iterations = 0;
    unsigned short threads = 0;
    unsigned on_off = 0;
};

// Reference usage line (gol-main.c:45), including its trailing " \n".
extern const char* const kUsage;

// Returns false when argc != 6 (caller prints kUsage and exits 255, like the reference).
bool parse_cli(int argc, const char* const* argv, CliArgs& out);

// Extension knobs (all optional).  Defaults reproduce the reference contract with a correct torus.
struct Options {
    std::string backend = "auto";   // GOL_BACKEND   auto | hip | cpu
    bool global_mode = false;       // GOL_GLOBAL    1: worldSize is the global board side (strong scaling)
    std::string decomp = "1d";      // GOL_DECOMP    1d | 2d | auto
    std::string grid = "";          // GOL_GRID      PxxPy, e.g. 4x2
    int halo_depth = 0;             // GOL_HALO_DEPTH generations per halo exchange (0 = auto)
    int kernel_depth = 0;           // GOL_KERNEL_DEPTH generations per kernel pass (0 = auto)
    bool graph = true;              // GOL_GRAPH     capture supersteps into hipGraphs
    bool overlap = true;            // GOL_OVERLAP   interior compute overlapped with the halo exchange
    u64 seed = 0x5EED;              // GOL_SEED      pattern 5 seed
    bool compat = false;            // GOL_COMPAT=reference: reproduce the reference's halo quirks
    int nranks = 0;                 // GOL_NRANKS    thread-mode rank count (single process)
    std::string transport = "auto"; // GOL_TRANSPORT auto | rccl | host (staged through host memory)
    std::string metrics_json = "";  // GOL_METRICS_JSON path for per-run metrics
    bool profile = false;           // GOL_PROFILE   per-phase hipEvent timing + roctx ranges
    i64 rows_per_wave = 0;          // GOL_ROWS_PER_WAVE segment height override (0 = auto)
    int waves_target = 0;           // GOL_WAVES     target wave count per sweep (0 = auto)
    std::string fault = "";         // GOL_FAULT     rank:gen fault injection (abort path testing)
    i64 checkpoint_every = 0;       // GOL_CHECKPOINT_EVERY generations between snapshots (0 = off)
    std::string checkpoint_path = "gol_ckpt";  // GOL_CHECKPOINT_PATH prefix of snapshot files
    std::string restart = "";       // GOL_RESTART   snapshot prefix to resume from
    double watchdog_s = 0;          // GOL_WATCHDOG  seconds before a stuck exchange aborts (0 = off)
    bool verbose = false;           // GOL_VERBOSE   log configuration to stderr
};

Options options_from_env();

}  // namespace gol
