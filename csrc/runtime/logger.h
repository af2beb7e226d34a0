// logger.h - the native runtime's logger (libVeles inc/veles/logger.h,
// src/logger.cc): per-domain, levelled, thread-safe lines on stderr.
//   VELES_RT_LOG=debug|info|warning|error|off   (default: warning)
// Use through the macros: VR_DBG / VR_INF / VR_WRN / VR_ERR(logger, fmt, ...)
#pragma once
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>

namespace veles_rt {

enum class LogLevel { Debug = 0, Info = 1, Warning = 2, Error = 3, Off = 4 };

inline LogLevel ParseLogLevel(const char* s) {
  if (!s || !*s) return LogLevel::Warning;
  if (!std::strcmp(s, "debug")) return LogLevel::Debug;
  if (!std::strcmp(s, "info")) return LogLevel::Info;
  if (!std::strcmp(s, "warning")) return LogLevel::Warning;
  if (!std::strcmp(s, "error")) return LogLevel::Error;
  if (!std::strcmp(s, "off")) return LogLevel::Off;
  return LogLevel::Warning;
}

class Logger {
 public:
  explicit Logger(std::string domain) : domain_(std::move(domain)) {}
  const std::string& domain() const { return domain_; }
  static LogLevel& Threshold() {
    static LogLevel lvl = ParseLogLevel(std::getenv("VELES_RT_LOG"));
    return lvl;
  }
  // where lines go (tests redirect it to a file); nullptr = stderr
  static FILE*& Sink() {
    static FILE* f = nullptr;
    return f;
  }
  bool Enabled(LogLevel l) const { return l >= Threshold(); }
  void Log(LogLevel l, const char* fmt, ...) const
      __attribute__((format(printf, 3, 4))) {
    if (!Enabled(l)) return;
    static const char* kNames[] = {"DEBUG", "INFO", "WARNING", "ERROR"};
    char msg[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(msg, sizeof(msg), fmt, ap);
    va_end(ap);
    char ts[32];
    std::time_t t = std::time(nullptr);
    std::tm tmv;
    localtime_r(&t, &tmv);
    std::strftime(ts, sizeof(ts), "%H:%M:%S", &tmv);
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    FILE* out = Sink() ? Sink() : stderr;
    std::fprintf(out, "%s %s %s: %s\n", ts, kNames[(int)l], domain_.c_str(),
                 msg);
    std::fflush(out);
  }

 private:
  std::string domain_;
};

#define VR_DBG(lg, ...) (lg).Log(::veles_rt::LogLevel::Debug, __VA_ARGS__)
#define VR_INF(lg, ...) (lg).Log(::veles_rt::LogLevel::Info, __VA_ARGS__)
#define VR_WRN(lg, ...) (lg).Log(::veles_rt::LogLevel::Warning, __VA_ARGS__)
#define VR_ERR(lg, ...) (lg).Log(::veles_rt::LogLevel::Error, __VA_ARGS__)

}  // namespace veles_rt
