#include "log.h"

#include <cstdio>
#include <mutex>

namespace mp {

namespace {
std::mutex g_mu;
int g_level = LOG_INFO;
FILE* g_file = nullptr;
bool g_stderr = true;
std::function<void(const std::string&)> g_cb;
}  // namespace

void log_set_level(int level) { std::lock_guard<std::mutex> l(g_mu); g_level = level; }
int log_level() { return g_level; }
void log_set_stderr(bool on) { std::lock_guard<std::mutex> l(g_mu); g_stderr = on; }

void log_set_file(const std::string& path) {
  std::lock_guard<std::mutex> l(g_mu);
  if (g_file) { fclose(g_file); g_file = nullptr; }
  if (!path.empty()) g_file = fopen(path.c_str(), "a");
}

void log_set_callback(std::function<void(const std::string&)> cb) {
  std::lock_guard<std::mutex> l(g_mu);
  g_cb = std::move(cb);
}

void logf(int level, const char* fmt, ...) {
  if (level < g_level) return;
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(buf, sizeof(buf) - 2, fmt, ap);
  va_end(ap);
  if (n < 0) return;
  if (n > (int)sizeof(buf) - 2) n = sizeof(buf) - 2;
  if (n == 0 || buf[n - 1] != '\n') { buf[n++] = '\n'; buf[n] = 0; }
  std::lock_guard<std::mutex> l(g_mu);
  if (g_stderr) { fputs(buf, stderr); fflush(stderr); }
  if (g_file) { fputs(buf, g_file); fflush(g_file); }
  if (g_cb) g_cb(std::string(buf, n));
}

}  // namespace mp
