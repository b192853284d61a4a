// gol-mi355x: roctx binding (see trace.hpp).
#include "gol/trace.hpp"

#include <dlfcn.h>

#include <cstdio>
#include <mutex>

#include "gol/common.hpp"

namespace gol {
namespace trace {

namespace {

struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    void (*mark)(const char*) = nullptr;
    bool ok = false;
};

const Roctx& roctx() {
    static Roctx r;
    static std::once_flag once;
    std::call_once(once, [] {
        if (env_int("GOL_ROCTX", env_int("GOL_PROFILE", 0)) == 0) return;
        void* h = nullptr;
        for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                                 "libroctx64.so"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) {
            fprintf(stderr, "[gol] GOL_ROCTX: no roctx library found; ranges disabled\n");
            return;
        }
        r.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
        r.pop = (int (*)())dlsym(h, "roctxRangePop");
        r.mark = (void (*)(const char*))dlsym(h, "roctxMarkA");
        r.ok = r.push && r.pop && r.mark;
    });
    return r;
}

}  // namespace

bool enabled() { return roctx().ok; }
void push(const char* name) {
    if (roctx().ok) roctx().push(name);
}
void pop() {
    if (roctx().ok) roctx().pop();
}
void mark(const char* name) {
    if (roctx().ok) roctx().mark(name);
}

}  // namespace trace
}  // namespace gol
