// gol-mi355x: roctx ranges for rocprofv3 (--marker-trace) and an optional stderr phase log.
//
// The reference has no instrumentation besides two MPI_Wtime calls on rank 0 around the whole
// loop (gol-main.c:82, 122).  Here the host side of every phase (init, superstep, exchange, graph
// launch, dump, checkpoint) is bracketed by a roctx range, so a marker trace lines the host
// schedule up with the kernel trace.  The roctx library is loaded with dlopen on first use, only
// when GOL_ROCTX=1 (or GOL_PROFILE=1); otherwise a Range costs one branch.
#pragma once

namespace gol {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

class Range {
   public:
    explicit Range(const char* name) : on_(enabled()) {
        if (on_) push(name);
    }
    ~Range() {
        if (on_) pop();
    }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;

   private:
    bool on_;
};

}  // namespace trace
}  // namespace gol
