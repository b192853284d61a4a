// gol-mi355x: Python bindings (pybind11) — module `_gol`.
//
// Exposes the native framework to the Python package (game-of-life---mpi-cuda_amd/): geometry,
// patterns, the work planner, transports (including a callback transport driven by
// torch.distributed / gloo), the Engine, dump formatting, the CLI driver and benchmark helpers.
// Engine.run releases the GIL; the callback transport re-acquires it for each call.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "gol/bench.hpp"
#include "gol/bits.hpp"
#include "gol/config.hpp"
#include "gol/cpu.hpp"
#include "gol/engine.hpp"
#include "gol/io.hpp"
#include "gol/pattern.hpp"
#include "gol/plan.hpp"
#include "gol/runtime.hpp"
#include "gol/transport.hpp"

namespace py = pybind11;
using namespace gol;

namespace {

// Transport whose primitives are Python callables (used with torch.distributed gloo on CPU).
//   send(peer, memoryview)              blocking, per-pair FIFO
//   recv(peer, memoryview)              fills the memoryview in place
//   exchange(sends, recvs) [optional]   lists of (peer, memoryview); must not deadlock
//   barrier() [optional]
class PyTransport : public Transport {
   public:
    PyTransport(int rank, int size, py::function send, py::function recv, py::object exchange, py::object barrier)
        : rank_(rank), size_(size), send_(std::move(send)), recv_(std::move(recv)), exch_(std::move(exchange)),
          barrier_(std::move(barrier)) {}
    ~PyTransport() override {
        py::gil_scoped_acquire g;
        send_ = py::function();
        recv_ = py::function();
        exch_ = py::object();
        barrier_ = py::object();
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    std::string name() const override { return "python"; }
    void send_bytes(int peer, const void* buf, size_t n) override {
        py::gil_scoped_acquire g;
        send_(peer, py::memoryview::from_memory(const_cast<void*>(buf), (ssize_t)n, true));
    }
    void recv_bytes(int peer, void* buf, size_t n) override {
        py::gil_scoped_acquire g;
        recv_(peer, py::memoryview::from_memory(buf, (ssize_t)n, false));
    }
    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void* s) override {
        py::gil_scoped_acquire g;
        if (exch_.is_none()) {
            py::gil_scoped_release r;
            Transport::exchange(sends, recvs, s);
            return;
        }
        py::list ls, lr;
        for (const Message& m : sends) ls.append(py::make_tuple(m.peer, py::memoryview::from_memory(m.buf, (ssize_t)m.bytes, true)));
        for (const Message& m : recvs) lr.append(py::make_tuple(m.peer, py::memoryview::from_memory(m.buf, (ssize_t)m.bytes, false)));
        exch_(ls, lr);
    }
    void barrier() override {
        {
            py::gil_scoped_acquire g;
            if (!barrier_.is_none()) {
                barrier_();
                return;
            }
        }
        Transport::barrier();
    }

   private:
    int rank_, size_;
    py::function send_, recv_;
    py::object exch_, barrier_;
};

py::array_t<u64> words_to_numpy(const std::vector<u64>& w, i64 rows, i64 nw) {
    py::array_t<u64> a({(py::ssize_t)rows, (py::ssize_t)nw});
    std::memcpy(a.mutable_data(), w.data(), w.size() * 8);
    return a;
}

py::dict stats_dict(const EngineStats& s) {
    py::dict d;
    d["generations"] = s.generations;
    d["supersteps"] = s.supersteps;
    d["exchanges"] = s.exchanges;
    d["halo_bytes"] = s.halo_bytes;
    d["graph_launches"] = s.graph_launches;
    d["depth"] = s.depth;
    d["plan_waves"] = s.plan_waves;
    d["lane_efficiency"] = s.lane_efficiency;
    d["predicted_us_per_gen"] = s.predicted_us_per_gen;
    d["predicted_gens"] = s.predicted_gens;
    d["t_exchange_ms"] = s.t_exchange_ms;
    d["t_compute_ms"] = s.t_compute_ms;
    d["kernel"] = s.kernel;
    d["schedule"] = s.schedule;
    d["kernel_depth"] = s.kernel_depth;
    d["tile_waves"] = s.tile_waves;
    d["tuning"] = s.tuning;
    d["registered"] = s.registered;
    return d;
}

}  // namespace

PYBIND11_MODULE(_gol, m) {
    m.doc() = "gol-mi355x native core (gfx950 HIP kernels, RCCL halo exchange, CPU backend)";

    py::register_exception<ContractError>(m, "ContractError");
    py::register_exception<Error>(m, "GolError");

    // ---- geometry -------------------------------------------------------------------------
    py::class_<Decomposition>(m, "Decomposition")
        .def_readonly("H", &Decomposition::H)
        .def_readonly("W", &Decomposition::W)
        .def_readonly("P", &Decomposition::P)
        .def_readonly("Px", &Decomposition::Px)
        .def_readonly("Py", &Decomposition::Py)
        .def_readonly("per_rank", &Decomposition::per_rank)
        .def_readonly("row_starts", &Decomposition::row_starts)
        .def_readonly("col_starts", &Decomposition::col_starts)
        .def_readonly("strip_starts", &Decomposition::strip_starts)
        .def("two_d", &Decomposition::two_d)
        .def("describe", &Decomposition::describe);
    m.def("make_decomposition", &make_decomposition, py::arg("N"), py::arg("P"), py::arg("global_mode") = false,
          py::arg("decomp") = "1d", py::arg("grid") = "", py::arg("width") = 0);

    py::class_<Geometry>(m, "Geometry")
        .def_readonly("dec", &Geometry::dec)
        .def_readonly("rank", &Geometry::rank)
        .def_readonly("cx", &Geometry::cx)
        .def_readonly("cy", &Geometry::cy)
        .def_readonly("row0", &Geometry::row0)
        .def_readonly("col0", &Geometry::col0)
        .def_readonly("h", &Geometry::h)
        .def_readonly("w", &Geometry::w)
        .def_property_readonly("nbr", [](const Geometry& g) { return std::vector<int>(g.nbr.begin(), g.nbr.end()); });
    m.def("make_geometry", &make_geometry);

    py::class_<Layout>(m, "Layout")
        .def(py::init<i64, i64, int>())
        .def_readonly("h", &Layout::h)
        .def_readonly("w", &Layout::w)
        .def_readonly("nw", &Layout::nw)
        .def_readonly("R", &Layout::R)
        .def_readonly("pitch", &Layout::pitch);
    m.def("clamp_halo_depth", &clamp_halo_depth);

    // ---- patterns -------------------------------------------------------------------------
    py::enum_<Fill>(m, "Fill").value("Zero", Fill::Zero).value("Ones", Fill::Ones).value("Random", Fill::Random);
    py::class_<PatternSpec>(m, "PatternSpec")
        .def(py::init<>())
        .def_readwrite("pattern", &PatternSpec::pattern)
        .def_readwrite("seed", &PatternSpec::seed)
        .def_readwrite("fill", &PatternSpec::fill)
        .def_readwrite("cells", &PatternSpec::cells);
    m.def("make_pattern", &make_pattern, py::arg("pattern"), py::arg("dec"), py::arg("seed") = 0x5EED);
    m.def("random_word", &random_word);
    m.def("mix64", &mix64);

    // ---- planner --------------------------------------------------------------------------
    m.def(
        "build_plan",
        [](const std::vector<std::tuple<i64, i64, i64, i64>>& regions, i64 nw, i64 h, i64 rows, int k, bool xwrap,
           bool fold) {
            std::vector<Region> rg;
            for (auto& t : regions) rg.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
            PlanStats st;
            std::vector<LaneDesc> lanes = build_plan(rg, nw, h, rows, k, xwrap, &st, kWavesPerBlock, 8, fold);
            py::array_t<i32> a({(py::ssize_t)lanes.size(), (py::ssize_t)4});
            std::memcpy(a.mutable_data(), lanes.data(), lanes.size() * sizeof(LaneDesc));
            py::dict d;
            d["waves"] = st.waves;
            d["active_lanes"] = st.active_lanes;
            d["lane_rows"] = st.lane_rows;
            d["out_words"] = st.out_words;
            return py::make_tuple(a, d);
        },
        py::arg("regions"), py::arg("nw"), py::arg("h"), py::arg("rows_per_chunk"), py::arg("k"),
        py::arg("xwrap") = false, py::arg("fold") = false);
    m.def("choose_rows_per_chunk", [](const std::vector<std::tuple<i64, i64, i64, i64>>& regions, int k, i64 target,
                                      i64 min_rows) {
        std::vector<Region> rg;
        for (auto& t : regions) rg.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
        return choose_rows_per_chunk(rg, k, target, min_rows);
    });

    // ---- transports -----------------------------------------------------------------------
    py::class_<Transport, std::shared_ptr<Transport>>(m, "Transport")
        .def("rank", &Transport::rank)
        .def("size", &Transport::size)
        .def("name", &Transport::name)
        .def("device_buffers", &Transport::device_buffers)
        .def("data_plane_ranks", &Transport::data_plane_ranks)
        .def("barrier", &Transport::barrier, py::call_guard<py::gil_scoped_release>())
        .def("allreduce_max", &Transport::allreduce_max, py::call_guard<py::gil_scoped_release>())
        .def("allreduce_min", &Transport::allreduce_min, py::call_guard<py::gil_scoped_release>())
        .def("allreduce_sum", &Transport::allreduce_sum, py::call_guard<py::gil_scoped_release>());
    py::class_<SelfTransport, Transport, std::shared_ptr<SelfTransport>>(m, "SelfTransport").def(py::init<>());
    py::class_<ThreadTransport, Transport, std::shared_ptr<ThreadTransport>>(m, "ThreadTransport");
    m.def("make_thread_transports", [](int P) {
        auto g = make_thread_group(P);
        std::vector<std::shared_ptr<Transport>> v;
        for (int r = 0; r < P; ++r) v.push_back(std::make_shared<ThreadTransport>(g, r));
        return v;
    });
    m.def("make_p2p_transports", [](int P) {
        auto g = make_thread_group(P);
        std::vector<std::shared_ptr<Transport>> v;
        for (int r = 0; r < P; ++r) v.push_back(make_p2p_emulation_transport(std::make_shared<ThreadTransport>(g, r)));
        return v;
    });
    py::class_<PyTransport, Transport, std::shared_ptr<PyTransport>>(m, "PyTransport")
        .def(py::init<int, int, py::function, py::function, py::object, py::object>(), py::arg("rank"),
             py::arg("size"), py::arg("send"), py::arg("recv"), py::arg("exchange") = py::none(),
             py::arg("barrier") = py::none());
    m.def("make_tcp_transport", &make_tcp_transport, py::arg("rank"), py::arg("size"), py::arg("addr"),
          py::arg("port"), py::arg("timeout_s") = 120.0, py::call_guard<py::gil_scoped_release>());
    m.def("make_rccl_transport", &make_rccl_transport, py::call_guard<py::gil_scoped_release>());
    m.def(
        "make_rccl_transport_with_id",
        [](std::shared_ptr<Transport> ctl, py::bytes uid) {
            std::string s = uid;
            py::gil_scoped_release r;
            return make_rccl_transport_with_id(ctl, s);
        },
        py::arg("control"), py::arg("unique_id"));
    m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });

    // ---- engine ---------------------------------------------------------------------------
    py::class_<EngineConfig>(m, "EngineConfig")
        .def(py::init<>())
        .def_readwrite("backend", &EngineConfig::backend)
        .def_readwrite("halo_depth", &EngineConfig::halo_depth)
        .def_readwrite("overlap", &EngineConfig::overlap)
        .def_readwrite("graph", &EngineConfig::graph)
        .def_readwrite("compat", &EngineConfig::compat)
        .def_readwrite("device", &EngineConfig::device)
        .def_readwrite("rows_per_wave", &EngineConfig::rows_per_wave)
        .def_readwrite("waves_target", &EngineConfig::waves_target)
        .def_readwrite("kernel", &EngineConfig::kernel)
        .def_readwrite("transport", &EngineConfig::transport)
        .def_readwrite("profile", &EngineConfig::profile)
        .def_readwrite("graph_supersteps", &EngineConfig::graph_supersteps)
        .def_readwrite("run_hint", &EngineConfig::run_hint)
        .def_readwrite("subtiles", &EngineConfig::subtiles)
        .def_readwrite("watchdog_s", &EngineConfig::watchdog_s)
        .def_readwrite("tile_waves", &EngineConfig::tile_waves)
        .def_readwrite("tune_tile_waves", &EngineConfig::tune_tile_waves)
        .def_readwrite("sub_occ", &EngineConfig::sub_occ)
        .def_readwrite("subtile_overlap", &EngineConfig::subtile_overlap)
        .def_readwrite("self_exchange", &EngineConfig::self_exchange)
        .def_readwrite("force_split", &EngineConfig::force_split)
        .def_readwrite("sched", &EngineConfig::sched)
        .def_readwrite("kernel_depth", &EngineConfig::kernel_depth)
        .def_readwrite("graph_rccl", &EngineConfig::graph_rccl)
        .def_readwrite("plan_xcds", &EngineConfig::plan_xcds);

    py::class_<Engine>(m, "Engine")
        .def_static(
            "create",
            [](const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) {
                py::gil_scoped_release r;
                return Engine::create(g, c, t);
            },
            py::arg("geometry"), py::arg("config"), py::arg("transport"))
        .def("init", &Engine::init, py::call_guard<py::gil_scoped_release>())
        .def("run", &Engine::run, py::call_guard<py::gil_scoped_release>())
        .def("synchronize", &Engine::synchronize, py::call_guard<py::gil_scoped_release>())
        .def("gpu_idle", &Engine::gpu_idle)
        .def("tile_words",
             [](Engine& e) {
                 std::vector<u64> w;
                 {
                     py::gil_scoped_release r;
                     w = e.tile_words();
                 }
                 return words_to_numpy(w, e.layout().h, e.layout().nw);
             })
        .def("set_tile_words",
             [](Engine& e, py::array_t<u64, py::array::c_style | py::array::forcecast> a) {
                 std::vector<u64> w(a.data(), a.data() + a.size());
                 py::gil_scoped_release r;
                 e.set_tile_words(w);
             })
        .def("local_reduce", &Engine::local_reduce, py::call_guard<py::gil_scoped_release>())
        .def("population", &Engine::population, py::call_guard<py::gil_scoped_release>())
        .def("fingerprint", &Engine::fingerprint, py::call_guard<py::gil_scoped_release>())
        .def("device_barrier", &Engine::device_barrier, py::call_guard<py::gil_scoped_release>())
        .def("phase_probe", &Engine::phase_probe, py::arg("k"), py::call_guard<py::gil_scoped_release>())
        .def("time_runs", &Engine::time_runs, py::arg("gens"), py::arg("reps"), py::call_guard<py::gil_scoped_release>())
        .def_property_readonly("geometry", &Engine::geometry)
        .def_property_readonly("layout", &Engine::layout)
        .def_property_readonly("generation", &Engine::generation)
        .def("stats", [](const Engine& e) { return stats_dict(e.stats()); })
        .def("describe", &Engine::describe)
        .def("backend_name", &Engine::backend_name)
        .def("halo_items", [](const Engine& e, int k) {
            py::list l;
            for (const auto& it : e.halo_items(k))
                l.append(py::make_tuple(dir_name(it.d), it.send_peer, it.recv_peer,
                                        py::make_tuple(it.send.r0, it.send.rows, it.send.c0, it.send.words),
                                        py::make_tuple(it.recv.r0, it.recv.rows, it.recv.c0, it.recv.words),
                                        it.contiguous));
            return l;
        });
    m.def("write_dumps", [](Engine& e, const std::string& path) {
        FILE* f = fopen(path.c_str(), "w");
        if (!f) throw Error("cannot open " + path);
        {
            py::gil_scoped_release r;
            write_dumps(e, f);
        }
        fclose(f);
    });
    m.def("save_checkpoint", &save_checkpoint, py::call_guard<py::gil_scoped_release>());
    m.def("load_checkpoint", &load_checkpoint, py::call_guard<py::gil_scoped_release>());

    // ---- CPU oracle ---------------------------------------------------------------------------
    m.def(
        "cpu_torus_step",
        [](py::array_t<u64, py::array::c_style | py::array::forcecast> words, i64 w, int gens) {
            // Full-torus reference on dense packed words (h x nw) via the CPU backend.
            const i64 h = words.shape(0), nw = words.shape(1);
            Layout L(h, w, 1);
            std::vector<u64> a((size_t)L.words(), 0), b((size_t)L.words(), 0);
            cpu::insert_words(a.data(), L, words.data());
            u64* cur = a.data();
            u64* oth = b.data();
            {
                py::gil_scoped_release r;
                for (int g = 0; g < gens; ++g) {
                    cpu::fill_ghost_cols_wrap(cur, L, 0, L.h);
                    cpu::fill_ghost_rows_wrap(cur, L);
                    cpu::step_rows(cur, oth, L, 0, L.h);
                    std::swap(cur, oth);
                }
            }
            std::vector<u64> out((size_t)(h * nw));
            cpu::extract_words(cur, L, out.data());
            return words_to_numpy(out, h, nw);
        },
        py::arg("words"), py::arg("w"), py::arg("gens"));

    // ---- I/O + CLI ------------------------------------------------------------------------
    m.def("dump_filename", &io::dump_filename);
    m.def("dump_header", &io::dump_header);
    m.def("format_rows", [](py::array_t<u64, py::array::c_style | py::array::forcecast> words, i64 w, i64 label0) {
        return py::bytes(io::format_rows(words.data(), words.shape(0), w, words.shape(1), label0));
    });
    m.def("timing_line", &io::timing_line);
    m.attr("BANNER") = std::string(io::kBanner);
    m.attr("USAGE") = std::string(kUsage);
    m.def("run_cli", [](std::vector<std::string> args) {
        std::vector<char*> argv;
        for (auto& s : args) argv.push_back(&s[0]);
        argv.push_back(nullptr);
        py::gil_scoped_release r;
        int rc = run_cli((int)args.size(), argv.data());
        fflush(stdout);
        return rc;
    });

    // ---- devices / bench ------------------------------------------------------------------
    m.def("hip_device_count", []() { return hip_device_count(nullptr); });
    m.def("hip_set_device", &hip_set_device);
    m.def(
        "naive_byte_run",
        [](i64 N, int gens, int threads, bool sync_each, u64 seed) {
            u64 pop = 0;
            double t;
            {
                py::gil_scoped_release r;
                t = bench::naive_byte_run(N, gens, threads, sync_each, seed, &pop);
            }
            return py::make_tuple(t, pop);
        },
        py::arg("N"), py::arg("gens"), py::arg("threads") = 256, py::arg("sync_each") = true,
        py::arg("seed") = 0x5EED);
    m.def("step_depth_supported", [](int k) { return k >= 1 && k <= 64; });
}
