// Minimal HTTP/1.1 server: thread per connection, Content-Length bodies, CORS, SSE streaming.
// (Reference: single-threaded blocking server, dllama-api.cpp:42-237, 331-368 - defect Q4.)
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "tcp.h"

namespace dl {

struct HttpRequest {
    std::string method, path, version;
    std::map<std::string, std::string> headers;  // lower-case keys
    std::string body;
};

class HttpConnection {
  public:
    explicit HttpConnection(Socket &&s) : sock_(std::move(s)) {}
    bool readRequest(HttpRequest &req);
    void writeResponse(int status, const std::string &contentType, const std::string &body);
    void writeJson(int status, const std::string &body) { writeResponse(status, "application/json; charset=utf-8", body); }
    void beginSse();
    void writeSse(const std::string &data);  // one "data: ..." event
    Socket &socket() { return sock_; }

  private:
    Socket sock_;
    std::string buf_;
};

using HttpHandler = std::function<void(const HttpRequest &, HttpConnection &)>;

class HttpServer {
  public:
    explicit HttpServer(int port) : server_(port) {}
    void route(const std::string &method, const std::string &path, HttpHandler h);
    void serveForever();  // blocks; one detached thread per connection
    int activeConnections() const { return active_.load(); }

  private:
    void handle(Socket s);
    ServerSocket server_;
    std::vector<std::tuple<std::string, std::string, HttpHandler>> routes_;
    std::atomic<int> active_{0};
};

}  // namespace dl
