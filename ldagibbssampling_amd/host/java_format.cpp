// java_format.cpp — see java_format.hpp.
#include "java_format.hpp"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace lda_host {

std::string java_double(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
  char buf[64];
  // shortest digits that round-trip, as d.ddde[+-]XX
  auto r = std::to_chars(buf, buf + sizeof(buf), std::fabs(x), std::chars_format::scientific);
  *r.ptr = '\0';
  std::string digits;
  const char* p = buf;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') digits.push_back(*p);
  const int exp10 = std::atoi(p + 1);  // value = d.ddd * 10^exp10
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = x < 0 ? "-" : "";
  const double ax = std::fabs(x);
  if (ax >= 1e-3 && ax < 1e7) {
    const int point = exp10 + 1;  // digits before the decimal point
    if (point <= 0) {
      out += "0.";
      out.append((size_t)(-point), '0');
      out += digits;
    } else if (point >= (int)digits.size()) {
      out += digits;
      out.append((size_t)(point - (int)digits.size()), '0');
      out += ".0";
    } else {
      out += digits.substr(0, (size_t)point);
      out += ".";
      out += digits.substr((size_t)point);
    }
  } else {
    out += digits[0];
    out += ".";
    out += digits.size() > 1 ? digits.substr(1) : std::string("0");
    out += "E";
    out += std::to_string(exp10);
  }
  return out;
}

std::string java_number5(double x) {
  if (std::isnan(x)) return "NaN";                 // DecimalFormatSymbols.getNaN()
  if (std::isinf(x)) return x > 0 ? "∞" : "-∞";
  // glibc rounds to the requested digits on the exact binary value with
  // round-half-even, which is DecimalFormat's HALF_EVEN on the exact double
  std::vector<char> buf(400);
  std::snprintf(buf.data(), buf.size(), "%.5f", x);
  std::string s(buf.data());
  bool neg = false;
  if (!s.empty() && s[0] == '-') {
    neg = true;
    s.erase(0, 1);
  }
  const size_t dot = s.find('.');
  std::string ip = s.substr(0, dot), fp = dot == std::string::npos ? "" : s.substr(dot + 1);
  while (!fp.empty() && fp.back() == '0') fp.pop_back();
  std::string grouped;
  const int n = (int)ip.size();
  for (int i = 0; i < n; ++i) {
    grouped.push_back(ip[(size_t)i]);
    const int rest = n - 1 - i;
    if (rest > 0 && rest % 3 == 0) grouped.push_back(',');
  }
  std::string out = neg ? "-" : "";
  out += grouped;
  if (!fp.empty()) {
    out += ".";
    out += fp;
  }
  return out;
}

}  // namespace lda_host
