// gol-mi355x: launch/bootstrap + the reference-compatible CLI driver (see runtime.hpp).
//
// Reference program flow (gol-main.c:30-146): argc check -> atoi -> MPI_Init -> fopen dump file ->
// gol_initMaster (device select + pattern) -> timer -> generation loop -> MPI_Barrier -> rank-0
// report -> banner -> dump -> MPI_Finalize -> free.  The same order is kept here, with two
// documented deviations: a barrier before the timer starts (fairer, never slower), and fatal errors
// abort every rank instead of leaving the others hanging (survey Q8, Q11).
#include "gol/runtime.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <exception>
#include <fstream>
#include <thread>

#include <fcntl.h>
#include <unistd.h>

#include "gol/io.hpp"
#include "gol/pattern.hpp"
#include "gol/trace.hpp"

namespace gol {

namespace {

double wtime() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int env_rank_var(const char* const* names, int dflt) {
    for (const char* const* n = names; *n; ++n) {
        const char* v = getenv(*n);
        if (v && *v) return atoi(v);
    }
    return dflt;
}

}  // namespace

LaunchInfo detect_launch(const Options& o) {
    LaunchInfo li;
    static const char* mpi_rank[] = {"PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK", nullptr};
    static const char* mpi_size[] = {"PMI_SIZE", "OMPI_COMM_WORLD_SIZE", nullptr};
    static const char* mpi_local[] = {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "PMI_LOCAL_RANK", nullptr};
    static const char* tr_rank[] = {"RANK", nullptr};
    static const char* tr_size[] = {"WORLD_SIZE", nullptr};
    static const char* tr_local[] = {"LOCAL_RANK", nullptr};
    if (o.nranks > 1) {
        li.mode = "threads";
        li.size = o.nranks;
        return li;
    }
    if (mpi_launched()) {
        li.mode = "mpi";
        li.rank = env_rank_var(mpi_rank, 0);
        li.size = env_rank_var(mpi_size, 1);
        li.local_rank = env_rank_var(mpi_local, li.rank);
        return li;
    }
    if (getenv("WORLD_SIZE") && atoi(getenv("WORLD_SIZE")) > 1) {
        li.mode = "tcp";
        li.rank = env_rank_var(tr_rank, 0);
        li.size = env_rank_var(tr_size, 1);
        li.local_rank = env_rank_var(tr_local, li.rank);
        return li;
    }
    return li;
}

std::shared_ptr<Transport> make_control_transport(const LaunchInfo& li, int* argc, char*** argv) {
    if (li.mode == "mpi") {
        auto t = make_mpi_transport(argc, argv);
        if (!t) throw Error("launched under mpirun but this build has no MPI support (GOL_WITH_MPI)");
        return t;
    }
    if (li.mode == "tcp") {
        std::string addr = env_str("MASTER_ADDR", "127.0.0.1");
        int port = (int)env_int("MASTER_PORT", 29500);
        return make_tcp_transport(li.rank, li.size, addr, port);
    }
    return std::make_shared<SelfTransport>();
}

std::string select_backend(const Options& o, int rank, int local_rank) {
    std::string b = o.backend;
    if (b == "cpu") return b;
    int err = 0;
    int n = hip_device_count(&err);
    if (b == "auto") {
        if (n <= 0) return "cpu";
        b = "hip";
    }
    if (b != "hip") throw Error("GOL_BACKEND must be auto, hip or cpu (got " + b + ")");
    if (n <= 0)
        throw ContractError(strprintf(" Unable to determine cuda device count, error is %d, count is %d\n", err, n), 255);
    int dev = (local_rank >= 0 ? local_rank : rank) % n;
    // the real hipError_t, as the reference prints its cudaError_t (gol-with-cuda.cu:298-299)
    if (const int e = hip_try_set_device(dev))
        throw ContractError(strprintf(" Unable to have rank %d set to cuda device %d, error is %d \n", rank, dev, e),
                            255);
    return b;
}

// True when every rank drives a different GPU (RCCL needs one rank per device; the reference's
// `rank % deviceCount` oversubscription, gol-with-cuda.cu:296, puts several ranks on one GPU).
static bool devices_distinct(Transport& control, int device) {
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    const std::string me = strprintf("%s#%d", host, device);
    std::vector<std::vector<u8>> all;
    control.gatherv(me.data(), me.size(), &all, 0);
    u8 ok = 1;
    if (control.rank() == 0) {
        std::vector<std::string> ids;
        for (auto& v : all) ids.emplace_back(v.begin(), v.end());
        std::sort(ids.begin(), ids.end());
        ok = std::adjacent_find(ids.begin(), ids.end()) == ids.end() ? 1 : 0;
    }
    control.broadcast(&ok, 1, 0);
    return ok != 0;
}

std::shared_ptr<Transport> make_data_transport(std::shared_ptr<Transport> control, const std::string& backend,
                                               const Options& o, int device) {
    if (backend != "hip" || control->size() == 1 || o.transport == "host") return control;
    if (o.transport == "p2p") return make_p2p_emulation_transport(control);  // RCCL semantics, one GPU
    if (!devices_distinct(*control, device)) {
        if (o.transport == "rccl")
            throw Error("GOL_TRANSPORT=rccl needs one rank per GPU, but ranks share a device");
        if (control->rank() == 0 && o.verbose)
            fprintf(stderr, "[gol] ranks share GPUs: halos are staged through host memory\n");
        return control;
    }
    return make_rccl_transport(control);
}

// threadsPerBlock (CLI argument 4): the reference's CUDA block size, which also decided whether its
// launch failed (blocks = W*H/T, T > 1024 invalid; survey Q6).  Here it is validated and used as a
// hint only: the workgroup size of the LDS tile kernel (T/64 waves; 512 -> 8, the default), unless
// GOL_TILE_WAVES is set.  Invalid values warn on stderr and keep the default.
void apply_threads_hint(EngineConfig& c, unsigned threads, bool report) {
    if (getenv("GOL_TILE_WAVES")) return;
    const bool ok = threads >= 64 && threads <= 1024 && threads % 64 == 0;
    if (!ok) {
        if (report)
            fprintf(stderr, "[gol] threadsPerBlock=%u is not a multiple of 64 in 64..1024; using the default "
                            "workgroup size\n", threads);
        return;
    }
    const int waves = (int)threads / 64;
    c.tile_waves = waves >= 16 ? 16 : (waves >= 8 ? 8 : 4);
}

EngineConfig engine_config(const Options& o, const std::string& backend, int device) {
    EngineConfig c;
    c.backend = backend;
    c.halo_depth = o.halo_depth;
    c.kernel_depth = o.kernel_depth;
    c.overlap = o.overlap;
    c.graph = o.graph;
    c.compat = o.compat;
    c.device = device;
    c.rows_per_wave = o.rows_per_wave;
    c.waves_target = o.waves_target;
    c.kernel = env_str("GOL_KERNEL", "auto");
    c.tile_waves = (int)env_int("GOL_TILE_WAVES", 8);
    c.tune_tile_waves = getenv("GOL_TILE_WAVES") == nullptr;
    c.transport = (o.transport == "rccl" || o.transport == "p2p") ? "device" : o.transport;
    c.profile = o.profile;
    c.graph_supersteps = (int)env_int("GOL_GRAPH_SUPERSTEPS", 0);
    c.subtiles = env_str("GOL_SUBTILES", "auto") == "auto" ? -1 : (int)env_int("GOL_SUBTILES", 0);
    c.watchdog_s = o.watchdog_s;
    c.sub_occ = (int)env_int("GOL_SUB_OCC", 2);
    auto tri = [](const char* name) {  // 0 off, 1 on, auto (default) -1: a timed candidate
        return env_str(name, "auto") == "auto" ? -1 : (int)(env_int(name, 0) != 0);
    };
    c.subtile_overlap = env_str("GOL_SUBTILE_OVERLAP", "auto") == "auto" ? -1 : (int)env_int("GOL_SUBTILE_OVERLAP", 0);
    c.self_exchange = env_int("GOL_SELF_EXCHANGE", 0) != 0;
    c.force_split = env_int("GOL_FORCE_SPLIT", 0) != 0;
    c.graph_rccl = tri("GOL_GRAPH_RCCL");
    c.plan_xcds = (int)env_int("GOL_PLAN_XCDS", 8);
    c.sched = env_str("GOL_SCHEDULE", "auto");
    if (c.sched != "auto" && c.sched != "split" && c.sched != "full")
        throw Error("GOL_SCHEDULE must be auto, split or full (got " + c.sched + ")");
    return c;
}

// ---------------------------------------------------------------------------------------------
// Dumps
// ---------------------------------------------------------------------------------------------

void write_dumps(Engine& eng, FILE* fp) {
    trace::Range range("gol.dump");
    const Geometry& g = eng.geometry();
    const Decomposition& d = g.dec;
    Transport& t = eng.transport();
    const int r = g.rank;
    io::write_header(fp, r);
    std::vector<u64> words = eng.tile_words();
    const i64 nw = eng.layout().nw;
    const bool tile_is_strip = d.Px == 1 && d.strip_starts[r] == g.row0 && d.strip_starts[r + 1] == g.row0 + g.h;
    bool all_strips = t.allreduce_min(tile_is_strip ? 1.0 : 0.0) > 0.5;
    if (all_strips) {
        io::write_rows(fp, words.data(), g.h, g.w, nw, g.row0);
        return;
    }
    // General case (2-D blocks): the dump of rank q is global rows strip_starts[q..q+1) at full width
    // (the reference's per-rank files, gol-main.c:17-28).  Every tile/strip overlap is one rectangle,
    // sent point to point from the tile's owner to the strip's owner in ONE exchange (no rank-0
    // funnel: each rank sends and receives only its own ~h x w cells).
    const i64 gw = g.global_words();
    const i64 s0 = d.strip_starts[r], s1 = d.strip_starts[r + 1];
    std::vector<u64> strip((size_t)((s1 - s0) * gw), 0);
    std::vector<std::vector<u64>> out_blocks, in_blocks;
    std::vector<Message> sends, recvs;
    struct InBlock {
        size_t idx;
        i64 r0, rows, word0, nwq;
    };
    std::vector<InBlock> ins;
    // what this rank's tile contributes to every strip
    for (int q = 0; q < d.P; ++q) {
        const i64 a = std::max(g.row0, d.strip_starts[q]), b = std::min(g.row0 + g.h, d.strip_starts[q + 1]);
        if (a >= b) continue;
        if (q == r) {
            for (i64 rr = a; rr < b; ++rr)
                memcpy(&strip[(size_t)((rr - s0) * gw + g.word0())], &words[(size_t)((rr - g.row0) * nw)],
                       (size_t)nw * 8);
            continue;
        }
        out_blocks.emplace_back(words.begin() + (a - g.row0) * nw, words.begin() + (b - g.row0) * nw);
    }
    size_t ob = 0;
    for (int q = 0; q < d.P; ++q) {
        const i64 a = std::max(g.row0, d.strip_starts[q]), b = std::min(g.row0 + g.h, d.strip_starts[q + 1]);
        if (a >= b || q == r) continue;
        sends.push_back({q, out_blocks[ob].data(), out_blocks[ob].size() * 8});
        ++ob;
    }
    // what every other rank's tile contributes to this rank's strip
    for (int q = 0; q < d.P; ++q) {
        if (q == r) continue;
        const Geometry gq = make_geometry(d, q);
        const i64 a = std::max(gq.row0, s0), b = std::min(gq.row0 + gq.h, s1);
        if (a >= b) continue;
        const i64 nwq = ceil_div(gq.w, 64);
        in_blocks.emplace_back((size_t)((b - a) * nwq));
        ins.push_back({in_blocks.size() - 1, a, b - a, gq.word0(), nwq});
        recvs.push_back({q, in_blocks.back().data(), in_blocks.back().size() * 8});
    }
    t.exchange_host(sends, recvs);
    for (const InBlock& ib : ins)
        for (i64 rr = 0; rr < ib.rows; ++rr)
            memcpy(&strip[(size_t)((ib.r0 - s0 + rr) * gw + ib.word0)], &in_blocks[ib.idx][(size_t)(rr * ib.nwq)],
                   (size_t)ib.nwq * 8);
    io::write_rows(fp, strip.data(), s1 - s0, d.W, gw, s0);
}

// ---------------------------------------------------------------------------------------------
// Checkpoints
// ---------------------------------------------------------------------------------------------
//
// One file per checkpoint, independent of the decomposition: a header, then the GLOBAL board as
// H rows of ceil(W/64) natural-order u64 words (bit b of word c = column 64c+b).  Every rank writes
// its own rectangle in place (pwrite at its rows' / words' offsets) and, on restart, reads its own
// rectangle whatever grid wrote the file: a snapshot taken by 8 ranks in 2-D resumes on 1 rank, or
// on 3 ranks in 1-D.  Rank 0 creates and sizes the file; the other ranks write after a barrier, and
// rank 0 renames it into place after a second one (a crash leaves only the .tmp file).

namespace {
struct CkptHeader {
    char magic[8];
    u64 version, H, W, words_per_row, generation, seed, reserved[2];
};
constexpr u64 kCkptVersion = 2;
std::string ckpt_name(const std::string& prefix) { return prefix + ".gol"; }

void pwrite_all(int fd, const void* buf, size_t n, off_t off, const std::string& name) {
    const char* p = (const char*)buf;
    while (n > 0) {
        const ssize_t w = pwrite(fd, p, n, off);
        if (w <= 0) throw Error("cannot write checkpoint " + name);
        p += w;
        n -= (size_t)w;
        off += w;
    }
}
void pread_all(int fd, void* buf, size_t n, off_t off, const std::string& name) {
    char* p = (char*)buf;
    while (n > 0) {
        const ssize_t got = pread(fd, p, n, off);
        if (got <= 0) throw Error("truncated checkpoint " + name);
        p += got;
        n -= (size_t)got;
        off += got;
    }
}
}  // namespace

void save_checkpoint(Engine& eng, const std::string& prefix, u64 seed) {
    trace::Range range("gol.checkpoint");
    const Geometry& g = eng.geometry();
    Transport& t = eng.transport();
    std::vector<u64> words = eng.tile_words();
    const i64 nw = eng.layout().nw, gw = g.global_words();
    const std::string name = ckpt_name(prefix), tmp = name + ".tmp";
    u8 ok = 1;
    if (g.rank == 0) {
        CkptHeader hd{};
        memcpy(hd.magic, "GOLCKPT2", 8);
        hd.version = kCkptVersion;
        hd.H = (u64)g.dec.H;
        hd.W = (u64)g.dec.W;
        hd.words_per_row = (u64)gw;
        hd.generation = eng.generation();
        hd.seed = seed;
        const int fd = open(tmp.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        ok = fd >= 0 && ftruncate(fd, (off_t)(sizeof(hd) + (size_t)(g.dec.H * gw) * 8)) == 0 &&
             pwrite(fd, &hd, sizeof(hd), 0) == (ssize_t)sizeof(hd);
        if (fd >= 0) close(fd);
    }
    t.broadcast(&ok, 1, 0);
    if (!ok) throw Error("cannot create checkpoint " + tmp);
    // Every rank writes its own rectangle into rank 0's file, so the file must be on a filesystem
    // shared by all ranks.  Failures are agreed on collectively (a rank that threw alone would leave
    // the others blocked in the next collective): every rank throws, or none does.
    std::string err;
    const int fd = open(tmp.c_str(), O_WRONLY);
    if (fd < 0) {
        err = strprintf("rank %d cannot open checkpoint %s created by rank 0 (checkpoints need a filesystem shared "
                        "by all ranks)",
                        g.rank, tmp.c_str());
    } else {
        try {
            const off_t base = (off_t)sizeof(CkptHeader);
            if (nw == gw) {  // full-width rows: one contiguous write
                pwrite_all(fd, words.data(), words.size() * 8, base + (off_t)(g.row0 * gw) * 8, tmp);
            } else {
                for (i64 r = 0; r < g.h; ++r)
                    pwrite_all(fd, &words[(size_t)(r * nw)], (size_t)nw * 8,
                               base + (off_t)((g.row0 + r) * gw + g.word0()) * 8, tmp);
            }
            if (fsync(fd) != 0) throw Error("cannot flush checkpoint " + tmp);
        } catch (const Error& e) {
            err = strprintf("rank %d: %s", g.rank, e.what());
        }
        close(fd);
    }
    if (t.allreduce_min(err.empty() ? 1.0 : 0.0) <= 0)
        throw Error(err.empty() ? "checkpoint " + tmp + " failed on another rank" : err);
    ok = 1;
    if (g.rank == 0) ok = rename(tmp.c_str(), name.c_str()) == 0;
    t.broadcast(&ok, 1, 0);
    if (!ok) throw Error("cannot rename checkpoint " + tmp + " to " + name);
}

u64 load_checkpoint(Engine& eng, const std::string& prefix) {
    const Geometry& g = eng.geometry();
    const std::string name = ckpt_name(prefix);
    const int fd = open(name.c_str(), O_RDONLY);
    if (fd < 0) throw Error("cannot open checkpoint " + name);
    CkptHeader hd{};
    const i64 nw = eng.layout().nw, gw = g.global_words();
    try {
        pread_all(fd, &hd, sizeof(hd), 0, name);
        if (memcmp(hd.magic, "GOLCKPT2", 8) != 0 || hd.version != kCkptVersion)
            throw Error("bad checkpoint header in " + name);
        if (hd.H != (u64)g.dec.H || hd.W != (u64)g.dec.W || hd.words_per_row != (u64)gw)
            throw Error(strprintf("checkpoint %s holds a %llux%llu board, this run has %lldx%lld", name.c_str(),
                                  (unsigned long long)hd.H, (unsigned long long)hd.W, (long long)g.dec.H,
                                  (long long)g.dec.W));
        std::vector<u64> words((size_t)(g.h * nw));
        const off_t base = (off_t)sizeof(CkptHeader);
        if (nw == gw) {
            pread_all(fd, words.data(), words.size() * 8, base + (off_t)(g.row0 * gw) * 8, name);
        } else {
            for (i64 r = 0; r < g.h; ++r)
                pread_all(fd, &words[(size_t)(r * nw)], (size_t)nw * 8,
                          base + (off_t)((g.row0 + r) * gw + g.word0()) * 8, name);
        }
        close(fd);
        eng.set_tile_words(words);
    } catch (...) {
        close(fd);
        throw;
    }
    return hd.generation;
}

// ---------------------------------------------------------------------------------------------
// CLI
// ---------------------------------------------------------------------------------------------

namespace {

struct RankResult {
    int status = 0;
};

void write_metrics(const Options& o, Engine& eng, const CliArgs& a, double duration, u64 gens, long updates,
                   const LaunchInfo& li) {
    if (o.metrics_json.empty() || eng.geometry().rank != 0) return;
    const EngineStats& s = eng.stats();
    const Decomposition& d = eng.geometry().dec;
    std::ofstream f(o.metrics_json);
    f << "{\n";
    f << "  \"metric\": \"cell-updates/sec\",\n";
    f << "  \"cell_updates_per_sec\": " << (duration > 0 ? (double)updates / duration : 0.0) << ",\n";
    f << "  \"duration_s\": " << duration << ",\n";
    f << "  \"cell_updates\": " << updates << ",\n";
    f << "  \"generations\": " << gens << ",\n";
    f << "  \"pattern\": " << a.pattern << ",\n  \"world_size\": " << a.world_size << ",\n";
    f << "  \"ranks\": " << d.P << ",\n  \"grid\": \"" << d.Px << "x" << d.Py << "\",\n";
    f << "  \"board\": [" << d.H << ", " << d.W << "],\n";
    f << "  \"mode\": \"" << (d.per_rank ? "per-rank" : "global") << "\",\n";
    f << "  \"launch\": \"" << li.mode << "\",\n";
    f << "  \"backend\": \"" << eng.backend_name() << "\",\n";
    f << "  \"transport\": \"" << eng.transport().name() << "\",\n";
    f << "  \"halo_depth\": " << s.depth << ",\n";
    f << "  \"kernel_depth\": " << s.kernel_depth << ",\n";
    f << "  \"supersteps\": " << s.supersteps << ",\n  \"exchanges\": " << s.exchanges << ",\n";
    f << "  \"halo_bytes_rank0\": " << s.halo_bytes << ",\n";
    f << "  \"graph_launches\": " << s.graph_launches << ",\n";
    f << "  \"kernel\": \"" << s.kernel << "\",\n";
    f << "  \"schedule\": \"" << s.schedule << "\",\n";
    f << "  \"autotune\": \"" << s.tuning << "\",\n";
    f << "  \"plan_waves\": " << s.plan_waves << ",\n  \"lane_efficiency\": " << s.lane_efficiency << ",\n";
    f << "  \"predicted_us_per_gen\": " << s.predicted_us_per_gen << ",\n";
    f << "  \"t_exchange_ms\": " << s.t_exchange_ms << ",\n  \"t_compute_ms\": " << s.t_compute_ms << "\n";
    f << "}\n";
}

int run_rank(const CliArgs& a, const Options& o, const LaunchInfo& li, std::shared_ptr<Transport> control) {
    const int rank = control->rank(), P = control->size();
    FILE* fp = nullptr;
    if (a.on_off == 1) {
        std::string fname = io::dump_filename(rank, P);
        fp = fopen(fname.c_str(), "w");
        if (!fp) {
            printf("ERROR IN RANK %d", rank);
            fflush(stdout);
            control->abort(255);
        }
    }
    try {
        const int local = li.mode == "threads" ? rank : li.local_rank;
        std::string backend = select_backend(o, rank, local);
        int device = -1;
        if (backend == "hip") {
            int n = hip_device_count();
            device = local % n;
            hip_set_device(device);  // before RCCL init: the communicator binds the current device
        }
        Decomposition dec = make_decomposition((i64)a.world_size, P, o.global_mode, o.decomp, o.grid);
        Geometry g = make_geometry(dec, rank);
        PatternSpec pat = make_pattern(a.pattern, dec, o.seed);
        std::shared_ptr<Transport> t = make_data_transport(control, backend, o, device);
        EngineConfig ec = engine_config(o, backend, device);
        apply_threads_hint(ec, a.threads, rank == 0);
        ec.run_hint = o.checkpoint_every > 0 ? (u64)o.checkpoint_every : (u64)a.iterations;
        std::unique_ptr<Engine> eng = Engine::create(g, ec, t);
        if (o.verbose && rank == 0) fprintf(stderr, "[gol] %s\n", eng->describe().c_str());
        eng->init(pat);
        u64 done = 0;
        if (!o.restart.empty()) done = load_checkpoint(*eng, o.restart);
        const u64 total = a.iterations;
        const u64 todo = done >= total ? 0 : total - done;

        t->barrier();
        const double t0 = wtime();
        if (o.checkpoint_every > 0) {
            u64 left = todo;
            while (left > 0) {
                u64 chunk = std::min<u64>(left, (u64)o.checkpoint_every);
                eng->run(chunk);
                left -= chunk;
                save_checkpoint(*eng, o.checkpoint_path, o.seed);
            }
        } else {
            eng->run(todo);
        }
        eng->synchronize();
        t->barrier();
        const double duration = wtime() - t0;
        const long updates = (long)P * (long)g.h * (long)g.w * (long)todo;
        // Reference formula counts P * N * N * iterations (gol-main.c:124-125): in per-rank mode and
        // 1-D that is exactly sum over ranks of h*w*iterations; use the global count in general.
        const long count = (long)dec.H * (long)dec.W * (long)todo;
        (void)updates;
        if (rank == 0) {
            std::string line = io::timing_line(duration, count);
            fwrite(line.data(), 1, line.size(), stdout);
            fputs(io::kBanner, stdout);
            fflush(stdout);
        }
        write_metrics(o, *eng, a, duration, todo, count, li);
        if (fp) {
            write_dumps(*eng, fp);
            fclose(fp);
            fp = nullptr;
        }
        t->barrier();
        return 0;
    } catch (const ContractError& e) {
        fputs(e.what(), stdout);
        fflush(stdout);
        if (fp) fclose(fp);
        if (P > 1) control->abort(e.exit_status);
        return e.exit_status;
    }
}

}  // namespace

int run_cli(int argc, char** argv) {
    CliArgs a;
    if (!parse_cli(argc, argv, a)) {
        printf("%s", kUsage);
        fflush(stdout);
        return 255;  // exit(-1), before any communicator (gol-main.c:43-47)
    }
    try {
        Options o = options_from_env();
        LaunchInfo li = detect_launch(o);
        if (li.mode == "threads") {
            auto group = make_thread_group(li.size);
            std::vector<int> status((size_t)li.size, 0);
            std::vector<std::thread> th;
            for (int r = 0; r < li.size; ++r) {
                th.emplace_back([&, r] {
                    try {
                        auto t = std::make_shared<ThreadTransport>(group, r);
                        status[(size_t)r] = run_rank(a, o, li, t);
                    } catch (const std::exception& e) {
                        fprintf(stderr, "[gol] rank %d: %s\n", r, e.what());
                        fflush(stderr);
                        const int code = thread_group_abort_code(*group);
                        _exit(code ? code : 1);
                    }
                });
            }
            for (auto& x : th) x.join();
            for (int s : status)
                if (s) return s;
            return 0;
        }
        auto control = make_control_transport(li, &argc, &argv);
        int st = 0;
        try {
            st = run_rank(a, o, li, control);
        } catch (const std::exception& e) {
            fprintf(stderr, "[gol] rank %d: %s\n", control->rank(), e.what());
            fflush(stderr);
            if (control->size() > 1) control->abort(1);
            return 1;
        }
        return st;
    } catch (const std::exception& e) {
        fprintf(stderr, "[gol] %s\n", e.what());
        return 1;
    }
}

}  // namespace gol
