// RFC3339 / RFC3339Nano time handling shared by the observation store, the
// metrics parser and the trial runtime.
//
// Semantics follow Go's time package as used by the reference:
//   * parsing: time.Parse(time.RFC3339Nano, s) (file-metricscollector.go:88,
//     mysql.go:74) - "YYYY-MM-DDTHH:MM:SS[.fffffffff](Z|+hh:mm|-hh:mm)";
//   * formatting: t.UTC().Format(time.RFC3339Nano) - fractional part with
//     trailing zeros removed, "Z" suffix (mysql.go:150).
// Times are (seconds since 1970, nanoseconds) pairs so that year 0001 (the
// "zero" timestamp the collector emits, time.Time{}.UTC()) is representable.
#pragma once
#include <cstdint>
#include <string>

namespace katib {

struct Timestamp {
  int64_t sec = 0;
  int32_t nsec = 0;
  bool operator<(const Timestamp& o) const { return sec < o.sec || (sec == o.sec && nsec < o.nsec); }
  bool operator>(const Timestamp& o) const { return o < *this; }
  bool operator<=(const Timestamp& o) const { return !(o < *this); }
  bool operator>=(const Timestamp& o) const { return !(*this < o); }
  bool operator==(const Timestamp& o) const { return sec == o.sec && nsec == o.nsec; }
};

// days since 1970-01-01 for a proleptic Gregorian civil date (H. Hinnant).
inline int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<int64_t>(doe) - 719468;
}

inline void civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = static_cast<unsigned>(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = static_cast<int64_t>(yoe) + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y += (m <= 2);
}

inline bool parse_digits(const std::string& s, size_t pos, size_t n, int64_t& out) {
  if (pos + n > s.size()) return false;
  int64_t v = 0;
  for (size_t i = 0; i < n; ++i) {
    char c = s[pos + i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  out = v;
  return true;
}

// Strict RFC3339Nano parse. Returns false if `s` is not a valid timestamp.
inline bool parse_rfc3339(const std::string& s, Timestamp& out) {
  int64_t Y, Mo, D, h, mi, se;
  if (s.size() < 20) return false;
  if (!parse_digits(s, 0, 4, Y) || s[4] != '-' || !parse_digits(s, 5, 2, Mo) || s[7] != '-' ||
      !parse_digits(s, 8, 2, D) || s[10] != 'T' || !parse_digits(s, 11, 2, h) || s[13] != ':' ||
      !parse_digits(s, 14, 2, mi) || s[16] != ':' || !parse_digits(s, 17, 2, se))
    return false;
  if (Mo < 1 || Mo > 12 || D < 1 || D > 31 || h > 23 || mi > 59 || se > 59) return false;
  static const int mdays[] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  int maxd = mdays[Mo - 1] - ((Mo == 2 && !leap) ? 1 : 0);
  if (D > maxd) return false;
  size_t p = 19;
  int64_t nsec = 0;
  if (p < s.size() && s[p] == '.') {
    ++p;
    size_t start = p;
    int64_t frac = 0;
    int nd = 0;
    while (p < s.size() && s[p] >= '0' && s[p] <= '9') {
      if (nd < 9) { frac = frac * 10 + (s[p] - '0'); ++nd; }
      ++p;
    }
    if (p == start) return false;
    while (nd < 9) { frac *= 10; ++nd; }
    nsec = frac;
  }
  if (p >= s.size()) return false;
  int64_t offset = 0;
  if (s[p] == 'Z') {
    ++p;
  } else if (s[p] == '+' || s[p] == '-') {
    int64_t oh, om;
    if (!parse_digits(s, p + 1, 2, oh) || p + 3 >= s.size() || s[p + 3] != ':' || !parse_digits(s, p + 4, 2, om))
      return false;
    if (oh > 23 || om > 59) return false;
    offset = (oh * 3600 + om * 60) * (s[p] == '-' ? -1 : 1);
    p += 6;
  } else {
    return false;
  }
  if (p != s.size()) return false;
  int64_t days = days_from_civil(Y, static_cast<unsigned>(Mo), static_cast<unsigned>(D));
  out.sec = days * 86400 + h * 3600 + mi * 60 + se - offset;
  out.nsec = static_cast<int32_t>(nsec);
  return true;
}

inline std::string format_rfc3339_nano(const Timestamp& t) {
  int64_t days = t.sec >= 0 ? t.sec / 86400 : -((-t.sec + 86399) / 86400);
  int64_t rem = t.sec - days * 86400;
  int64_t y;
  unsigned m, d;
  civil_from_days(days, y, m, d);
  char buf[64];
  int n = snprintf(buf, sizeof(buf), "%04lld-%02u-%02uT%02d:%02d:%02d", static_cast<long long>(y), m, d,
                   static_cast<int>(rem / 3600), static_cast<int>((rem / 60) % 60), static_cast<int>(rem % 60));
  std::string out(buf, n);
  if (t.nsec != 0) {
    char fb[16];
    snprintf(fb, sizeof(fb), "%09d", t.nsec);
    std::string frac(fb);
    while (!frac.empty() && frac.back() == '0') frac.pop_back();
    out += "." + frac;
  }
  out += "Z";
  return out;
}

inline Timestamp zero_time() {
  Timestamp t;
  t.sec = days_from_civil(1, 1, 1) * 86400;
  t.nsec = 0;
  return t;
}

inline const std::string& zero_time_str() {
  static const std::string z = "0001-01-01T00:00:00Z";
  return z;
}

}  // namespace katib
