#include <kungfu/http.hpp>
#include <kungfu/log.hpp>
#include <kungfu/transport.hpp>

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstring>
#include <sstream>
#include <stdexcept>

namespace kungfu {

namespace {

std::string lower(std::string s) {
    for (auto &c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    return s;
}

// Reads headers + body (by Content-Length).  Returns false on error.
// is_request: an HTTP/1.1 request without Content-Length has no body (a client such as
// urllib or curl keeps its write side open waiting for the response); a response
// without Content-Length is delimited by the connection close.
bool read_http(int fd, std::string *head, std::string *body, bool is_request) {
    std::string buf;
    char tmp[4096];
    size_t hend = std::string::npos;
    while (hend == std::string::npos) {
        ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
        if (n <= 0) return false;
        buf.append(tmp, static_cast<size_t>(n));
        hend = buf.find("\r\n\r\n");
        if (buf.size() > (1 << 20) && hend == std::string::npos) return false;
    }
    *head = buf.substr(0, hend);
    *body = buf.substr(hend + 4);
    size_t clen = 0;
    bool has_len = false;
    std::istringstream hs(*head);
    std::string line;
    while (std::getline(hs, line)) {
        auto c = line.find(':');
        if (c == std::string::npos) continue;
        if (lower(line.substr(0, c)) == "content-length") {
            clen = std::stoul(line.substr(c + 1));
            has_len = true;
        }
    }
    if (has_len) {
        while (body->size() < clen) {
            ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
            if (n <= 0) return false;
            body->append(tmp, static_cast<size_t>(n));
        }
        body->resize(clen);
    } else if (!is_request) {
        // read until close (responses without Content-Length)
        for (;;) {
            ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
            if (n <= 0) break;
            body->append(tmp, static_cast<size_t>(n));
        }
    }
    return true;
}

const char *status_text(int s) {
    switch (s) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 500: return "Internal Server Error";
    }
    return "Status";
}

}  // namespace

HttpServer::HttpServer(uint16_t port, Handler h, const std::string &bind_addr)
    : port_(port), bind_(bind_addr), h_(std::move(h)) {}

HttpServer::~HttpServer() { stop(); }

void HttpServer::start() {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons(port_);
    inet_pton(AF_INET, bind_.c_str(), &addr.sin_addr);
    if (::bind(fd_, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) != 0 || ::listen(fd_, 128) != 0) {
        int e = errno;
        ::close(fd_);
        fd_ = -1;
        throw std::runtime_error("http: cannot listen on port " + std::to_string(port_) + ": " + std::strerror(e));
    }
    if (port_ == 0) {
        socklen_t len = sizeof(addr);
        getsockname(fd_, reinterpret_cast<sockaddr *>(&addr), &len);
        port_ = ntohs(addr.sin_port);
    }
    th_ = std::thread([this] { loop(); });
}

void HttpServer::loop() {
    while (!stop_.load()) {
        pollfd p{fd_, POLLIN, 0};
        if (::poll(&p, 1, 200) <= 0) continue;
        int c = ::accept(fd_, nullptr, nullptr);
        if (c < 0) continue;
        std::lock_guard<std::mutex> lk(mu_);
        workers_.emplace_back([this, c] {
            timeval tv{30, 0};
            setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
            std::string head, body;
            HttpResponse resp;
            if (!read_http(c, &head, &body, /*is_request=*/true)) {
                ::close(c);
                return;
            }
            HttpRequest req;
            std::istringstream hs(head);
            std::string line, target;
            std::getline(hs, line);
            std::istringstream rl(line);
            rl >> req.method >> target;
            auto q = target.find('?');
            req.path = target.substr(0, q);
            if (q != std::string::npos) req.query = target.substr(q + 1);
            while (std::getline(hs, line)) {
                auto cp = line.find(':');
                if (cp == std::string::npos) continue;
                std::string v = line.substr(cp + 1);
                while (!v.empty() && (v[0] == ' ')) v.erase(0, 1);
                while (!v.empty() && (v.back() == '\r')) v.pop_back();
                req.headers[lower(line.substr(0, cp))] = v;
            }
            req.body = body;
            try {
                resp = h_(req);
            } catch (const std::exception &e) {
                resp.status = 500;
                resp.body = e.what();
            }
            std::ostringstream os;
            os << "HTTP/1.1 " << resp.status << " " << status_text(resp.status) << "\r\n"
               << "Content-Type: " << resp.content_type << "\r\n"
               << "Content-Length: " << resp.body.size() << "\r\n"
               << "Connection: close\r\n\r\n"
               << resp.body;
            std::string out = os.str();
            write_full(c, out.data(), out.size());
            ::shutdown(c, SHUT_WR);
            ::close(c);
        });
    }
}

void HttpServer::stop() {
    if (stop_.exchange(true)) return;
    if (th_.joinable()) th_.join();
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    std::vector<std::thread> ws;
    {
        std::lock_guard<std::mutex> lk(mu_);
        ws.swap(workers_);
    }
    for (auto &t : ws)
        if (t.joinable()) t.join();
}

int http_request(const std::string &method, const std::string &url, const std::string &body, std::string *resp,
                 double timeout_sec) {
    std::string rest = url;
    if (rest.rfind("http://", 0) == 0) rest = rest.substr(7);
    auto slash = rest.find('/');
    std::string hostport = rest.substr(0, slash), path = slash == std::string::npos ? "/" : rest.substr(slash);
    auto colon = hostport.rfind(':');
    std::string host = hostport.substr(0, colon);
    std::string port = colon == std::string::npos ? "80" : hostport.substr(colon + 1);
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return -1;
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    timeval tv{static_cast<long>(timeout_sec), static_cast<long>((timeout_sec - static_cast<long>(timeout_sec)) * 1e6)};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc != 0) {
        ::close(fd);
        return -1;
    }
    std::ostringstream os;
    os << method << " " << path << " HTTP/1.1\r\nHost: " << hostport << "\r\nContent-Length: " << body.size()
       << "\r\nContent-Type: application/json\r\nConnection: close\r\n\r\n"
       << body;
    std::string req = os.str();
    if (!write_full(fd, req.data(), req.size())) {
        ::close(fd);
        return -1;
    }
    std::string head, rbody;
    bool ok = read_http(fd, &head, &rbody, /*is_request=*/false);
    ::close(fd);
    if (!ok) return -1;
    int status = -1;
    std::istringstream hs(head);
    std::string proto;
    hs >> proto >> status;
    if (resp) *resp = rbody;
    return status;
}

}  // namespace kungfu
