// lda_guard.h — keeps C++ exceptions from crossing the C ABI (SURVEY.md §8b:
// "No C++ exception crosses the ABI").  Internal to liblda_mi355x.so.
//
// Every extern "C" entry point that can allocate runs its body through
// guarded(): std::bad_alloc becomes LDA_ERR_OUT_OF_MEMORY, any other
// exception LDA_ERR_INTERNAL, with the message in lda_last_error().  Host
// buffers whose size the caller controls come from host_vector(), which
// also honours the test hook lda_debug_fail_host_alloc (the n-th such
// allocation on this thread throws std::bad_alloc).
#pragma once
#include <exception>
#include <new>
#include <string>
#include <vector>

#include "../../include/lda_mi355x.h"

namespace lda_abi {

void set_error(const std::string& msg);   // lda_last_error's text (lda_capi.cpp)
void check_host_alloc();                  // throws std::bad_alloc when the hook fires

template <typename F>
lda_status guarded(F&& f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed (std::bad_alloc)");
    return LDA_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    set_error(std::string("internal error: ") + e.what());
    return LDA_ERR_INTERNAL;
  } catch (...) {
    set_error("internal error: unknown exception");
    return LDA_ERR_INTERNAL;
  }
}

template <typename T>
std::vector<T> host_vector(size_t n, const T& v = T()) {
  check_host_alloc();
  return std::vector<T>(n, v);
}

}  // namespace lda_abi
