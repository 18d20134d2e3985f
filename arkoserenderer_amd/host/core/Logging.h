// Logging.h — ARKOSE_LOG subset (arkcore/core/Logging.h:40-100): severity-tagged
// stdout lines; Fatal exits the process like the reference.
#pragma once

#include <cstdio>
#include <cstdlib>

namespace ark {
enum class LogLevel { Verbose, Info, Warning, Error, Fatal };
int& errorCounter();
const char* logLevelName(LogLevel);
} // namespace ark

#define ARKOSE_LOG(level, ...)                                                              \
    do {                                                                                    \
        std::fprintf(stderr, "[%s] ", ::ark::logLevelName(::ark::LogLevel::level));         \
        std::fprintf(stderr, __VA_ARGS__);                                                  \
        std::fputc('\n', stderr);                                                           \
        if (::ark::LogLevel::level == ::ark::LogLevel::Error) ++::ark::errorCounter();      \
        if (::ark::LogLevel::level == ::ark::LogLevel::Fatal) std::exit(13);                \
    } while (0)

#define ARKOSE_ASSERT(cond)                                                                 \
    do {                                                                                    \
        if (!(cond)) ARKOSE_LOG(Fatal, "assertion failed: %s (%s:%d)", #cond, __FILE__, __LINE__); \
    } while (0)
