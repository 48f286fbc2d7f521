// Host-only: step 1's alldata.json text from the rows as arrays (step1_proc2d.py:345-375 writes
// json.dump(alldata) of per-frame row lists [track id, x1, y1, x2, y2, [[x, y, score] x J], assigned id,
// id score]).  The text is byte for byte what Python's json.dumps gives for the same rows -- floats in
// Python's repr (the shortest round-trip digits, exponent form when the decimal exponent is < -4 or > 15,
// NaN / Infinity as json writes them), ", " between items -- so the files equal the reference's format
// and the Python mirror's, while the formatting runs without the interpreter lock (called from step 1's
// background writer through ctypes).
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "mq_hip.h"

#include <string>
extern int mq_fail_host(const std::string& msg, int code);

namespace {

struct Out {
  char* p;
  char* end;
  bool ok = true;
  void put(const char* s, size_t n) {
    if (p + n > end) {
      ok = false;
      return;
    }
    std::memcpy(p, s, n);
    p += n;
  }
  void put(const char* s) { put(s, std::strlen(s)); }
  void put(char c) { put(&c, 1); }
};

// Python float.__repr__ (PyOS_double_to_string(x, 'r', 0, Py_DTSF_ADD_DOT_0)) as json.dumps writes it
void put_pyfloat(Out& o, double x) {
  if (std::isnan(x)) return o.put("NaN");
  if (std::isinf(x)) return o.put(x > 0 ? "Infinity" : "-Infinity");
  if (x == 0.0) return o.put(std::signbit(x) ? "-0.0" : "0.0");
  char buf[40];
  const auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);  // shortest d.ddde+XX
  const char* s = buf;
  const char* e = r.ptr;
  bool neg = false;
  if (*s == '-') {
    neg = true;
    ++s;
  }
  char dig[24];
  int nd = 0;
  const char* q = s;
  for (; q < e && *q != 'e'; ++q)
    if (*q != '.') dig[nd++] = *q;
  int ex = 0;
  std::from_chars(q + 1 + (q[1] == '+' ? 1 : 0), e, ex);
  const int decpt = ex + 1;  // digits d1 d2 ... x 10^(decpt - nd)
  if (neg) o.put('-');
  if (decpt <= -4 || decpt > 16) {
    o.put(dig[0]);
    if (nd > 1) {
      o.put('.');
      o.put(dig + 1, nd - 1);
    }
    char eb[8];
    const int ee = decpt - 1;
    const int ae = ee < 0 ? -ee : ee;
    int n = 0;
    eb[n++] = 'e';
    eb[n++] = ee < 0 ? '-' : '+';
    if (ae >= 100) eb[n++] = char('0' + ae / 100);
    eb[n++] = char('0' + (ae / 10) % 10);
    eb[n++] = char('0' + ae % 10);
    o.put(eb, n);
  } else if (decpt <= 0) {
    o.put("0.");
    for (int i = 0; i < -decpt; ++i) o.put('0');
    o.put(dig, nd);
  } else if (decpt >= nd) {
    o.put(dig, nd);
    for (int i = nd; i < decpt; ++i) o.put('0');
    o.put(".0");
  } else {
    o.put(dig, decpt);
    o.put('.');
    o.put(dig + decpt, nd - decpt);
  }
}

void put_int(Out& o, int64_t v) {
  char buf[24];
  const auto r = std::to_chars(buf, buf + sizeof(buf), v);
  o.put(buf, r.ptr - buf);
}

}  // namespace

extern "C" int mq_alldata_json(int n_frames, const int32_t* nrows, const int64_t* tid, const double* box,
                               const double* kp, int J, const int64_t* assigned, const double* score, char* out,
                               int64_t cap, int64_t* len) {
  if (n_frames < 0 || J <= 0 || !out || !len || cap < 2 || (n_frames > 0 && !nrows))
    return mq_fail_host("mq_alldata_json: bad arguments", -1);
  Out o{out, out + cap};
  int64_t r = 0;
  o.put('[');
  for (int f = 0; f < n_frames; ++f) {
    if (f) o.put(", ");
    o.put('[');
    for (int i = 0; i < nrows[f]; ++i, ++r) {
      if (i) o.put(", ");
      o.put('[');
      put_int(o, tid[r]);
      for (int b = 0; b < 4; ++b) {
        o.put(", ");
        put_pyfloat(o, box[r * 4 + b]);
      }
      o.put(", [");
      for (int j = 0; j < J; ++j) {
        if (j) o.put(", ");
        o.put('[');
        const double* k = kp + (r * J + j) * 3;
        put_pyfloat(o, k[0]);
        o.put(", ");
        put_pyfloat(o, k[1]);
        o.put(", ");
        put_pyfloat(o, k[2]);
        o.put(']');
      }
      o.put("], ");
      put_int(o, assigned[r]);
      o.put(", ");
      put_pyfloat(o, score[r]);
      o.put(']');
    }
    o.put(']');
  }
  o.put(']');
  if (!o.ok) return mq_fail_host("mq_alldata_json: output buffer too small", -2);
  *len = o.p - out;
  return 0;
}
