#include "http.h"

#include <algorithm>
#include <cstdio>
#include <sstream>
#include <thread>
#include <tuple>

#include <sys/socket.h>

namespace dl {

static const char *kCors =
    "Access-Control-Allow-Origin: *\r\n"
    "Access-Control-Allow-Methods: GET, POST, OPTIONS\r\n"
    "Access-Control-Allow-Headers: Content-Type, Authorization\r\n";

static const char *statusText(int s) {
    switch (s) {
        case 200: return "OK";
        case 204: return "No Content";
        case 400: return "Bad Request";
        case 404: return "Not Found";
        case 405: return "Method Not Allowed";
        case 413: return "Payload Too Large";
        case 500: return "Internal Server Error";
        case 503: return "Service Unavailable";
        default: return "OK";
    }
}

bool HttpConnection::readRequest(HttpRequest &req) {
    // read headers
    size_t hdrEnd;
    char tmp[4096];
    while ((hdrEnd = buf_.find("\r\n\r\n")) == std::string::npos) {
        if (buf_.size() > (1u << 20)) throw NetError("headers too large");
        const ssize_t r = ::recv(sock_.fd(), tmp, sizeof(tmp), 0);
        if (r <= 0) return false;
        buf_.append(tmp, (size_t)r);
    }
    std::istringstream hs(buf_.substr(0, hdrEnd));
    std::string line;
    std::getline(hs, line);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    {
        std::istringstream ls(line);
        ls >> req.method >> req.path >> req.version;
    }
    if (req.method.empty()) throw NetError("bad request line");
    while (std::getline(hs, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const size_t c = line.find(':');
        if (c == std::string::npos) continue;
        std::string k = line.substr(0, c), v = line.substr(c + 1);
        std::transform(k.begin(), k.end(), k.begin(), ::tolower);
        v.erase(0, v.find_first_not_of(' '));
        req.headers[k] = v;
    }
    size_t len = 0;
    auto it = req.headers.find("content-length");
    if (it != req.headers.end()) len = (size_t)std::stoull(it->second);
    if (len > (64u << 20)) throw NetError("body too large");
    buf_.erase(0, hdrEnd + 4);
    while (buf_.size() < len) {
        const ssize_t r = ::recv(sock_.fd(), tmp, sizeof(tmp), 0);
        if (r <= 0) return false;
        buf_.append(tmp, (size_t)r);
    }
    req.body = buf_.substr(0, len);
    buf_.erase(0, len);
    // strip query string
    const size_t q = req.path.find('?');
    if (q != std::string::npos) req.path.resize(q);
    return true;
}

void HttpConnection::writeResponse(int status, const std::string &contentType, const std::string &body) {
    char head[512];
    const int n = std::snprintf(head, sizeof(head),
                                "HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %zu\r\n%sConnection: close\r\n\r\n",
                                status, statusText(status), contentType.c_str(), body.size(), kCors);
    sock_.sendAll(head, (u64)n);
    if (!body.empty()) sock_.sendAll(body.data(), body.size());
}

void HttpConnection::beginSse() {
    std::string head = "HTTP/1.1 200 OK\r\nContent-Type: text/event-stream\r\nCache-Control: no-cache\r\n";
    head += kCors;
    head += "Connection: close\r\n\r\n";
    sock_.sendAll(head.data(), head.size());
}

void HttpConnection::writeSse(const std::string &data) {
    const std::string ev = "data: " + data + "\r\n\r\n";
    sock_.sendAll(ev.data(), ev.size());
}

void HttpServer::route(const std::string &method, const std::string &path, HttpHandler h) {
    routes_.emplace_back(method, path, std::move(h));
}

void HttpServer::handle(Socket s) {
    active_++;
    try {
        HttpConnection conn(std::move(s));
        HttpRequest req;
        if (conn.readRequest(req)) {
            if (logLevel() >= 1) std::printf("🔷 %s %s\n", req.method.c_str(), req.path.c_str());
            std::fflush(stdout);
            if (req.method == "OPTIONS") {
                conn.writeResponse(204, "text/plain", "");
            } else {
                bool pathFound = false, served = false;
                for (auto &r : routes_) {
                    if (std::get<1>(r) != req.path) continue;
                    pathFound = true;
                    if (std::get<0>(r) != req.method) continue;
                    std::get<2>(r)(req, conn);
                    served = true;
                    break;
                }
                if (!served)
                    conn.writeJson(pathFound ? 405 : 404,
                                   pathFound ? "{\"error\":\"method not allowed\"}" : "{\"error\":\"not found\"}");
            }
        }
    } catch (const std::exception &e) {
        std::printf("Socket error: %s\n", e.what());
    }
    active_--;
}

void HttpServer::serveForever() {
    while (true) {
        Socket s = server_.accept();
        std::thread([this](Socket sock) { handle(std::move(sock)); }, std::move(s)).detach();
    }
}

}  // namespace dl
