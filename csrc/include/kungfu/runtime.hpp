// Process-global runtime accessors shared by the C ABI and the Python binding.
#pragma once

#include <kungfu/peer.hpp>

#include <memory>
#include <string>

namespace kungfu {

Peer *global_peer();
Peer &require_peer();
std::shared_ptr<Session> require_session();
void init_global_peer(const PeerConfig &cfg);
void finalize_global_peer();
void set_last_error(const std::string &e);

}  // namespace kungfu
