// Minimal HTTP/1.1 server and client used by the control plane: the config
// server (GET/PUT/POST/DELETE /config, /stop), the monitor's /metrics endpoint
// and the runner's debug endpoint.  One request per connection
// ("Connection: close"), thread per connection.
//
// Parity: srcs/go/kungfu/elastic/configserver/configserver.go:15-112 (REST API),
// srcs/go/monitor/server.go:15-30 (metrics HTTP), srcs/go/kungfu/runner/handler.go:117-123.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kungfu {

struct HttpRequest {
    std::string method, path, query, body;
    std::map<std::string, std::string> headers;
};

struct HttpResponse {
    int status = 200;
    std::string body;
    std::string content_type = "text/plain";
};

class HttpServer {
  public:
    using Handler = std::function<HttpResponse(const HttpRequest &)>;
    HttpServer(uint16_t port, Handler h, const std::string &bind_addr = "0.0.0.0");
    ~HttpServer();
    void start();  // throws if it cannot bind
    void stop();
    uint16_t port() const { return port_; }

  private:
    void loop();
    uint16_t port_;
    std::string bind_;
    Handler h_;
    int fd_ = -1;
    std::atomic<bool> stop_{false};
    std::thread th_;
    std::mutex mu_;
    std::vector<std::thread> workers_;
};

// url: http://host:port/path ; returns HTTP status (or -1 on connection error).
int http_request(const std::string &method, const std::string &url, const std::string &body, std::string *resp,
                 double timeout_sec = 10.0);

}  // namespace kungfu
