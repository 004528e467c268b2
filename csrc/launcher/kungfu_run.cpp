// kungfu-run: spawn one worker process per slot with the kungfu env contract.
#include "launcher.hpp"

int main(int argc, char **argv) { return kungfu::launcher::kungfu_run_main(argc, argv); }
