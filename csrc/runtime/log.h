// Logger (E13): levels, stderr sink, optional file sink (--log-file), optional callback sink
// (the orchestrator forwards log lines as SSE `log` events, reference `main.rs:63-80`).
#pragma once
#include <cstdarg>
#include <functional>
#include <string>

namespace mp {

enum LogLevel { LOG_DEBUG = 0, LOG_INFO = 1, LOG_WARN = 2, LOG_ERROR = 3 };

void log_set_level(int level);
int log_level();
void log_set_file(const std::string& path);       // "" closes
void log_set_stderr(bool on);
// callback receives fully formatted lines (with trailing '\n'); thread-safe
void log_set_callback(std::function<void(const std::string&)> cb);
void logf(int level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define MP_LOGD(...) ::mp::logf(::mp::LOG_DEBUG, __VA_ARGS__)
#define MP_LOGI(...) ::mp::logf(::mp::LOG_INFO, __VA_ARGS__)
#define MP_LOGW(...) ::mp::logf(::mp::LOG_WARN, __VA_ARGS__)
#define MP_LOGE(...) ::mp::logf(::mp::LOG_ERROR, __VA_ARGS__)

}  // namespace mp
