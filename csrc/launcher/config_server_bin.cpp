// kungfu-config-server: standalone elastic cluster config server (REST /config).
#include "launcher.hpp"

namespace kungfu {
namespace launcher {
int config_server_main(int argc, char **argv);
}
}  // namespace kungfu

int main(int argc, char **argv) { return kungfu::launcher::config_server_main(argc, argv); }
