// gol-mi355x: CLI + environment parsing (see config.hpp).
#include "gol/config.hpp"

#include <cstring>
#include <vector>

namespace gol {

const char* const kUsage =
    "GOL requires 5 arguments: pattern number, sq size of the world and the number of itterations, "
    "threads per block and output-on-off e.g. ./gol 0 32 2 512 0 \n";

bool parse_cli(int argc, const char* const* argv, CliArgs& out) {
    if (argc != 6) return false;
    // atoi + implicit conversions, exactly as gol-main.c:49-53
    out.pattern = (unsigned)atoi(argv[1]);
    out.world_size = (unsigned)atoi(argv[2]);
    out.iterations = (unsigned)atoi(argv[3]);
    out.threads = (unsigned short)atoi(argv[4]);
    out.on_off = (unsigned)atoi(argv[5]);
    return true;
}

std::string strprintf(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    va_list ap2;
    va_copy(ap2, ap);
    int n = vsnprintf(nullptr, 0, fmt, ap);
    va_end(ap);
    std::vector<char> buf((size_t)n + 1);
    vsnprintf(buf.data(), buf.size(), fmt, ap2);
    va_end(ap2);
    return std::string(buf.data(), (size_t)n);
}

std::string env_str(const char* name, const std::string& dflt) {
    const char* v = getenv(name);
    return (v && *v) ? std::string(v) : dflt;
}

long long env_int(const char* name, long long dflt) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    char* end = nullptr;
    long long x = strtoll(v, &end, 0);
    if (end == v) throw Error(strprintf("%s=%s is not an integer", name, v));
    return x;
}

bool env_flag(const char* name, bool dflt) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    std::string s(v);
    if (s == "1" || s == "true" || s == "yes" || s == "on") return true;
    if (s == "0" || s == "false" || s == "no" || s == "off") return false;
    throw Error(strprintf("%s=%s is not a boolean", name, v));
}

Options options_from_env() {
    Options o;
    o.backend = env_str("GOL_BACKEND", o.backend);
    o.global_mode = env_flag("GOL_GLOBAL", o.global_mode);
    o.decomp = env_str("GOL_DECOMP", o.decomp);
    o.grid = env_str("GOL_GRID", o.grid);
    o.halo_depth = (int)env_int("GOL_HALO_DEPTH", o.halo_depth);
    o.kernel_depth = (int)env_int("GOL_KERNEL_DEPTH", o.kernel_depth);
    o.graph = env_flag("GOL_GRAPH", o.graph);
    o.overlap = env_flag("GOL_OVERLAP", o.overlap);
    o.seed = (u64)env_int("GOL_SEED", (long long)o.seed);
    std::string compat = env_str("GOL_COMPAT", "");
    if (!compat.empty() && compat != "reference" && compat != "none")
        throw Error("GOL_COMPAT must be 'reference' or 'none' (got " + compat + ")");
    o.compat = compat == "reference";
    o.nranks = (int)env_int("GOL_NRANKS", 0);
    o.transport = env_str("GOL_TRANSPORT", o.transport);
    o.metrics_json = env_str("GOL_METRICS_JSON", "");
    o.profile = env_flag("GOL_PROFILE", false);
    o.rows_per_wave = env_int("GOL_ROWS_PER_WAVE", 0);
    o.waves_target = (int)env_int("GOL_WAVES", 0);
    o.fault = env_str("GOL_FAULT", "");
    o.checkpoint_every = env_int("GOL_CHECKPOINT_EVERY", 0);
    o.checkpoint_path = env_str("GOL_CHECKPOINT_PATH", o.checkpoint_path);
    o.restart = env_str("GOL_RESTART", "");
    o.watchdog_s = (double)env_int("GOL_WATCHDOG", 0);
    o.verbose = env_flag("GOL_VERBOSE", false);
    if (o.halo_depth < 0 || o.halo_depth > 128) throw Error("GOL_HALO_DEPTH must be in 1..128 (0 = auto)");
    if (o.kernel_depth < 0 || o.kernel_depth > 64) throw Error("GOL_KERNEL_DEPTH must be in 1..64 (0 = auto)");
    return o;
}

}  // namespace gol
