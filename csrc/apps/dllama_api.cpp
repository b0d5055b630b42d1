// `dllama-api` — OpenAI-style HTTP server over the multi-user scheduler
// (reference: src/dllama-api.cpp:250-410, src/api-types.hpp).
//
//   POST /v1/chat/completions  {"messages":[...], "max_tokens", "temperature", "top_p", "seed",
//                               "stop", "stream"}
//        -> {"generated_text": ...} (the reference/web-ui shape) plus the OpenAI
//           {"id","object","created","model","choices":[...],"usage":{...}} fields;
//           "stream": true -> server-sent events with chat.completion.chunk objects + [DONE]
//   GET  /v1/models            {"object":"list","data":[{"id":<model file name>, ...}]}
//   GET  /health               scheduler counters (JSON)
//   GET  /v1/metrics           the same counters in Prometheus text format
//   GET  /, /app.js, /style.css  the chat web UI (--web-ui <dir>, default ./web-ui when present)
// Requests run concurrently (thread per connection); the scheduler batches them into shared forwards.
#include <csignal>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <sstream>
#include <string>

#include "../net/http.h"
#include "../net/json.h"
#include "../runtime/scheduler.h"

using namespace dl;
using json::Value;

namespace {

std::string modelName(const AppArgs &a) {
    if (!a.synthetic.empty()) return a.synthetic;
    const size_t p = a.modelPath.find_last_of("/\\");
    return p == std::string::npos ? a.modelPath : a.modelPath.substr(p + 1);
}

struct Api {
    AppArgs args;
    InferenceSession *sess;
    Scheduler *sched;
    std::unique_ptr<ChatTemplateGenerator> tmpl;
    std::string model;
    std::atomic<u64> counter{0};

    std::vector<int> buildPrompt(const Value &messages) {
        std::vector<ChatItem> items;
        for (const Value &m : messages.items()) items.push_back(ChatItem{m["role"].asString(), m["content"].asString()});
        Tokenizer &tok = sess->tokenizer();
        if (tmpl) {
            GeneratedChat g = tmpl->generate(items, true);
            return tok.encode(g.content, true, true);
        }
        // reference behaviour when no chat template is available: "role: content\n" lines
        std::string flat;
        for (auto &it : items) flat += it.role + ": " + it.message + "\n";
        return tok.encode(flat, true, false);
    }

    void complete(const HttpRequest &req, HttpConnection &conn) {
        Value body;
        try {
            body = Value::parse(req.body);
            if (!body["messages"].isArray() || body["messages"].size() == 0) throw std::runtime_error("messages required");
        } catch (const std::exception &e) {
            Value err = Value::object();
            err.set("error", std::string("Invalid request: ") + e.what());
            conn.writeJson(400, err.dump());
            return;
        }
        GenParams p;
        p.temperature = args.temperature;
        p.topp = args.topp;
        p.seed = args.seed + counter.fetch_add(1);
        if (body["max_tokens"].isNumber()) p.maxTokens = (int)body["max_tokens"].asNumber();
        if (body["temperature"].isNumber()) p.temperature = (float)body["temperature"].asNumber();
        if (body["top_p"].isNumber()) p.topp = (float)body["top_p"].asNumber();
        if (body["seed"].isNumber()) p.seed = (u64)body["seed"].asNumber();
        if (body["stop"].isString()) p.stop.push_back(body["stop"].asString());
        if (body["stop"].isArray())
            for (const Value &s : body["stop"].items())
                if (s.isString()) p.stop.push_back(s.asString());
        const bool stream = body["stream"].isBool() && body["stream"].asBool();
        std::vector<int> prompt;
        try {
            prompt = buildPrompt(body["messages"]);
        } catch (const std::exception &e) {
            Value err = Value::object();
            err.set("error", std::string("Invalid messages: ") + e.what());
            conn.writeJson(400, err.dump());
            return;
        }
        const int promptTokens = (int)prompt.size();
        auto r = sched->submit(std::move(prompt), p);
        // if this handler unwinds early (client gone: a write throws), stop generating for it
        struct CancelOnExit {
            GenRequest *r;
            ~CancelOnExit() { r->cancel(); }
        } cancelGuard{r.get()};
        const std::string id = "chatcmpl-" + std::to_string(r->id);
        const long created = (long)std::time(nullptr);
        if (stream) {
            conn.beginSse();
            bool first = true;
            std::string d;
            while (r->nextDelta(d)) {
                Value chunk = Value::object();
                chunk.set("id", id);
                chunk.set("object", "chat.completion.chunk");
                chunk.set("created", created);
                chunk.set("model", model);
                Value ch = Value::object();
                ch.set("index", 0);
                Value delta = Value::object();
                if (first) delta.set("role", "assistant");
                delta.set("content", d);
                ch.set("delta", delta);
                ch.set("finish_reason", Value());
                chunk.set("choices", Value::array()).push(ch);
                conn.writeSse(chunk.dump());
                first = false;
            }
            Value chunk = Value::object();
            chunk.set("id", id);
            chunk.set("object", "chat.completion.chunk");
            chunk.set("created", created);
            chunk.set("model", model);
            Value ch = Value::object();
            ch.set("index", 0);
            ch.set("delta", Value::object());
            ch.set("finish_reason", r->finishReason);
            chunk.set("choices", Value::array()).push(ch);
            conn.writeSse(chunk.dump());
            conn.writeSse("[DONE]");
            return;
        }
        const std::string text = r->wait();
        if (r->finishReason == "error") {
            Value err = Value::object();
            err.set("error", r->error.empty() ? "generation failed" : r->error);
            conn.writeJson(500, err.dump());
            return;
        }
        Value resp = Value::object();
        resp.set("id", id);
        resp.set("object", "chat.completion");
        resp.set("created", created);
        resp.set("model", model);
        Value choice = Value::object();
        choice.set("index", 0);
        Value msg = Value::object();
        msg.set("role", "assistant");
        msg.set("content", text);
        choice.set("message", msg);
        choice.set("finish_reason", r->finishReason);
        resp.set("choices", Value::array()).push(choice);
        Value usage = Value::object();
        usage.set("prompt_tokens", promptTokens);
        usage.set("completion_tokens", r->completionTokens);
        usage.set("total_tokens", promptTokens + r->completionTokens);
        resp.set("usage", usage);
        resp.set("generated_text", text);
        conn.writeJson(200, resp.dump());
        if (logLevel() >= 1) {
            std::printf("🔶 %s: %d prompt + %d completion tokens (%s)\n", id.c_str(), promptTokens, r->completionTokens,
                        r->finishReason.c_str());
            std::fflush(stdout);
        }
    }

    void models(const HttpRequest &, HttpConnection &conn) {
        Value m = Value::object();
        m.set("id", model);
        m.set("object", "model");
        m.set("created", 0);
        m.set("owned_by", "user");
        Value list = Value::object();
        list.set("object", "list");
        list.set("data", Value::array()).push(m);
        conn.writeJson(200, list.dump());
    }

    // Prometheus text exposition of the scheduler counters (SURVEY §5.5 "GET /v1/metrics").
    void metrics(const HttpRequest &, HttpConnection &conn, int connections) {
        const SchedulerStats s = sched->stats();
        std::string out;
        auto metric = [&](const char *name, const char *type, const char *help, double v) {
            char line[256];
            std::snprintf(line, sizeof(line), "# HELP %s %s\n# TYPE %s %s\n%s %.17g\n", name, help, name, type, name, v);
            out += line;
        };
        metric("dllama_forwards_total", "counter", "Batched forward passes run by the scheduler.", (double)s.forwards);
        metric("dllama_rows_total", "counter", "Token rows processed (prefill + decode).", (double)s.rows);
        metric("dllama_prefill_rows_total", "counter", "Prompt token rows prefilled.", (double)s.prefillRows);
        metric("dllama_decode_rows_total", "counter", "Decode token rows.", (double)s.decodeRows);
        metric("dllama_requests_completed_total", "counter", "Finished requests.", (double)s.completed);
        metric("dllama_generated_tokens_total", "counter", "Tokens generated for finished requests.", (double)s.generatedTokens);
        metric("dllama_requests_cancelled_total", "counter", "Requests dropped after their client disconnected.",
               (double)s.cancelled);
        metric("dllama_busy_seconds_total", "counter", "Time spent in forward passes.", s.busyMs / 1000.0);
        metric("dllama_active_requests", "gauge", "Requests holding a KV slot.", (double)s.active);
        metric("dllama_queued_requests", "gauge", "Requests waiting for a KV slot.", (double)s.queued);
        metric("dllama_kv_slots", "gauge", "KV-cache slots (max concurrent sequences).", (double)sess->nSlots());
        metric("dllama_nodes", "gauge", "Tensor-parallel ranks.", (double)sess->nNodes());
        metric("dllama_http_connections", "gauge", "Open HTTP connections.", (double)connections);
        conn.writeResponse(200, "text/plain; version=0.0.4; charset=utf-8", out);
    }

    void health(const HttpRequest &, HttpConnection &conn) {
        SchedulerStats s = sched->stats();
        Value v = Value::object();
        v.set("status", "ok");
        v.set("model", model);
        v.set("backend", sess->isGpu() ? "hip" : "cpu");
        v.set("nodes", sess->nNodes());
        v.set("slots", sess->nSlots());
        v.set("active", s.active);
        v.set("queued", s.queued);
        v.set("forwards", (double)s.forwards);
        v.set("rows", (double)s.rows);
        v.set("prefill_rows", (double)s.prefillRows);
        v.set("decode_rows", (double)s.decodeRows);
        v.set("completed", (double)s.completed);
        v.set("cancelled", (double)s.cancelled);
        v.set("generated_tokens", (double)s.generatedTokens);
        v.set("busy_ms", s.busyMs);
        conn.writeJson(200, v.dump());
    }
};

bool readFile(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

void serveWebUi(HttpServer &server, const std::string &dir) {
    static const char *files[][3] = {{"/", "index.html", "text/html; charset=utf-8"},
                                     {"/app.js", "app.js", "application/javascript"},
                                     {"/style.css", "style.css", "text/css"}};
    for (auto &f : files) {
        const std::string path = dir + "/" + f[1], type = f[2];
        server.route("GET", f[0], [path, type](const HttpRequest &, HttpConnection &c) {
            std::string body;
            if (readFile(path, body))
                c.writeResponse(200, type, body);
            else
                c.writeJson(404, "{\"error\":\"web ui file missing\"}");
        });
    }
}

void usage() {
    std::fprintf(stderr,
                 "Usage: dllama-api {--model <path>} {--tokenizer <path>} [--port <p>]\n"
                 "        [--buffer-float-type {f32|f16|q40|q80}]\n"
                 "        [--max-seq-len <max>] [--slots <n>] [--max-batch <n>] [--prefill-chunk <n>]\n"
                 "        [--kv-pages <n> --kv-page-size <p>]   (GPU paged KV: slots share a page pool)\n"
                 "        [--nthreads <n>] [--gpu-index <i>]\n"
                 "        [--workers <ip:port> ...]\n"
                 "        [--temperature <temp>] [--topp <t>] [--seed <s>] [--chat-template <t>]\n"
                 "        [--web-ui <dir>] [--metrics <file|->]\n");
}

}  // namespace

int main(int argc, char **argv) {
#ifdef SIGPIPE
    std::signal(SIGPIPE, SIG_IGN);
#endif
    try {
        AppArgs args = AppArgs::parse(argc, argv, false);
        if (args.help) {
            usage();
            return 0;
        }
        InferenceSession sess(args, args.slots > 0 ? args.slots : 8);
        Api api;
        api.args = args;
        api.sess = &sess;
        api.model = modelName(args);
        ChatStops stops(sess.tokenizer());
        if (!stops.stops.empty() && (sess.tokenizer().hasChatTemplate() || args.chatTemplate != ChatTemplateType::UNKNOWN)) {
            try {
                api.tmpl.reset(new ChatTemplateGenerator(args.chatTemplate, sess.tokenizer().chatTemplate(), stops.stops[0]));
            } catch (const std::exception &e) {
                std::printf("⚠️  chat template unavailable (%s); using role-prefixed prompts\n", e.what());
            }
        }
        Scheduler sched(sess);
        api.sched = &sched;
        HttpServer server(args.port);
        server.route("POST", "/v1/chat/completions", [&](const HttpRequest &r, HttpConnection &c) { api.complete(r, c); });
        server.route("GET", "/v1/models", [&](const HttpRequest &r, HttpConnection &c) { api.models(r, c); });
        server.route("GET", "/health", [&](const HttpRequest &r, HttpConnection &c) { api.health(r, c); });
        server.route("GET", "/v1/metrics",
                     [&](const HttpRequest &r, HttpConnection &c) { api.metrics(r, c, server.activeConnections()); });
        std::string ui = args.webUi;
        std::string probe;
        if (ui.empty() && readFile("web-ui/index.html", probe)) ui = "web-ui";
        if (!ui.empty()) {
            serveWebUi(server, ui);
            std::printf("Web UI: http://127.0.0.1:%d/\n", args.port);
        }
        std::printf("Server URL: http://127.0.0.1:%d/v1/\n", args.port);
        std::fflush(stdout);
        server.serveForever();
    } catch (const std::exception &e) {
        std::printf("🚨 Critical error: %s\n", e.what());
        return 1;
    }
    return 0;
}
