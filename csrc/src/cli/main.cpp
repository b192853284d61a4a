// gol-mi355x: the `gol` executable.
//   ./gol <pattern> <worldSize> <iterations> <threadsPerBlock> <output_on_off>
// Same arguments, stdout lines, exit statuses and Rank_<r>_of_<P>.txt dumps as the reference
// (gol-main.c:30-146).  Extensions are GOL_* environment variables (config.hpp).
#include "gol/runtime.hpp"

int main(int argc, char** argv) { return gol::run_cli(argc, argv); }
