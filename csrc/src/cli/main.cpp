// gol-mi355x: the `gol` executable.
//   ./gol <pattern> <worldSize> <iterations> <threadsPerBlock> <output_on_off>
// Same arguments, stdout lines, exit statuses and Rank_<r>_of_<P>.txt dumps as the reference
// (gol-main.c:30-146).  Extensions are GOL_* environment variables (config.hpp).
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include "gol/runtime.hpp"

namespace {

// Fatal-signal report: the raw return addresses of the faulting thread (resolve them offline with
// `addr2line -e build/gol -f -C <addr - load base>`; the load base is the first r-xp line of the
// maps dump), then the default action.  Async-signal-safe calls only.
void on_fatal_signal(int sig) {
    static const char msg[] = "[gol] fatal signal; backtrace:\n";
    ssize_t w = write(STDERR_FILENO, msg, sizeof(msg) - 1);
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, STDERR_FILENO);
    const int fd = open("/proc/self/maps", 0);
    if (fd >= 0) {
        char buf[4096];
        ssize_t r;
        while ((r = read(fd, buf, sizeof(buf))) > 0) w = write(STDERR_FILENO, buf, (size_t)r);
        close(fd);
    }
    (void)w;
    signal(sig, SIG_DFL);
    raise(sig);
}

}  // namespace

int main(int argc, char** argv) {
    for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL}) signal(sig, on_fatal_signal);
    return gol::run_cli(argc, argv);
}
