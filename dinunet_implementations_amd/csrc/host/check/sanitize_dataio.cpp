// Host-code sanitizer driver for csrc/host/dataio.cpp (SURVEY.md §5.2 "debug target").
//
// Built together with dataio.cpp into one executable with -fsanitize=address,undefined (GPU
// AddressSanitizer is not available for gfx950 on this pool, so the sanitized target is the
// host runtime: file parsing, windowing, metrics).  Every entry point is driven through its
// edge cases -- CRLF / blank / trailing-whitespace lines, missing and malformed files, files
// with more values than requested, windows that end exactly at T, fp32 and fp64 sources, row
// subsets, tied ROC scores, absent classes -- and the results are checked against values
// computed here, so a pass means "no ASan/UBSan report AND correct answers".
// Exit status 0 = pass; any failure prints the check and returns 1 (sanitizer reports abort).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
long dnh_fs_load(const char* const* paths, long n, int nfeat, float* out, int threads);
int dnh_ica_windows(const void* src, int src_f64, long N, int C, int T, int W, int stride,
                    int temporal, const long* rows, long nrows, float* out, int threads);
double dnh_roc_auc(const double* scores, const long* labels, long n);
int dnh_confusion2(const long* pred, const long* labels, long n, long* out);
int dnh_version();
}

static int g_fail = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

static std::string write_file(const std::string& dir, const std::string& name,
                              const std::string& body) {
  const std::string p = dir + "/" + name;
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) { std::perror(p.c_str()); std::exit(2); }
  std::fwrite(body.data(), 1, body.size(), f);
  std::fclose(f);
  return p;
}

static void check_fs(const std::string& dir) {
  // many files so the OpenMP loop really runs in parallel (dynamic schedule, chunk 8)
  std::vector<std::string> paths;
  const int n = 64, nfeat = 5;
  for (int i = 0; i < n; ++i) {
    std::string body = "Measure:volume\tsubject" + std::to_string(i) + "\r\n";
    for (int k = 0; k < nfeat + (i % 3); ++k) {  // some files carry extra values
      body += "Region-" + std::to_string(k) + "\t" + std::to_string(1.0 + k + i) +
              ((k % 2) ? " \t\r\n" : "\n");
      if (k == 2) body += "\n   \n";  // blank / whitespace-only lines
    }
    if (i % 5 == 0) body.pop_back();  // no trailing newline
    paths.push_back(write_file(dir, "s" + std::to_string(i) + ".txt", body));
  }
  std::vector<const char*> cp;
  for (auto& p : paths) cp.push_back(p.c_str());
  std::vector<float> out((size_t)n * nfeat, -1.f);
  CHECK(dnh_fs_load(cp.data(), n, nfeat, out.data(), 4) == 0);
  for (int i = 0; i < n; ++i) {
    const double mx = nfeat + i;  // max of the first nfeat values 1+k+i
    for (int k = 0; k < nfeat; ++k)
      CHECK(out[(size_t)i * nfeat + k] == (float)((1.0 + k + i) / mx));
  }
  // error reporting: first failing index and kind
  const std::string shortf = write_file(dir, "short.txt", "hdr\nA\t1\n");
  const std::string badf = write_file(dir, "bad.txt", "hdr\nA\t1\nB\tnot_a_number\n");
  const std::string emptyf = write_file(dir, "empty.txt", "");
  const std::string missing = dir + "/does_not_exist.txt";
  std::vector<float> o2(4 * 2);
  {
    const char* p[] = {cp[0], shortf.c_str()};
    CHECK(dnh_fs_load(p, 2, 2, o2.data(), 2) == 1 + 1 * 4 + 3);
  }
  {
    const char* p[] = {badf.c_str(), cp[1]};
    CHECK(dnh_fs_load(p, 2, 2, o2.data(), 2) == 1 + 0 * 4 + 2);
  }
  {
    const char* p[] = {cp[0], cp[1], missing.c_str(), emptyf.c_str()};
    CHECK(dnh_fs_load(p, 4, 2, o2.data(), 3) == 1 + 2 * 4 + 1);
  }
  CHECK(dnh_fs_load(nullptr, 0, 2, o2.data(), 1) == 0);
  CHECK(dnh_fs_load(cp.data(), 1, 0, o2.data(), 1) == 1);
}

template <typename T>
static void check_windows_t(int f64) {
  const long N = 7;
  const int C = 3, Tn = 61, W = 5, stride = 3, temporal = 60;
  const int S = temporal / W;  // 12 windows, last ends at 11*3+5 = 38 <= 61
  std::vector<T> src((size_t)N * C * Tn);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (T)(0.25 * (double)i - 3.0);
  const long rows[] = {6, 0, 3, 3};
  const long nrows = 4;
  std::vector<float> out((size_t)nrows * S * C * W, -7.f);
  CHECK(dnh_ica_windows(src.data(), f64, N, C, Tn, W, stride, temporal, rows, nrows,
                        out.data(), 4) == 0);
  for (long i = 0; i < nrows; ++i)
    for (int j = 0; j < S; ++j)
      for (int c = 0; c < C; ++c)
        for (int w = 0; w < W; ++w) {
          const float got = out[(((size_t)i * S + j) * C + c) * W + w];
          const T ref = src[((size_t)rows[i] * C + c) * Tn + (size_t)j * stride + w];
          CHECK(got == (float)ref);
        }
  // all rows (rows == nullptr), windows ending exactly at T
  const int T2 = 20, W2 = 10;
  std::vector<T> s2((size_t)2 * C * T2);
  for (size_t i = 0; i < s2.size(); ++i) s2[i] = (T)i;
  std::vector<float> o2((size_t)2 * 2 * C * W2);
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, W2, W2, T2, nullptr, 2, o2.data(), 2) == 0);
  CHECK(o2.back() == (float)s2.back());
  // rejected arguments: window past T, row out of range, bad sizes
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, W2, 11, T2, nullptr, 2, o2.data(), 1) == 2);
  const long bad_rows[] = {0, 2};
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, W2, W2, T2, bad_rows, 2, o2.data(), 1) == 2);
  const long neg_rows[] = {-1};
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, W2, W2, T2, neg_rows, 1, o2.data(), 1) == 2);
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, 0, W2, T2, nullptr, 2, o2.data(), 1) == 1);
  CHECK(dnh_ica_windows(s2.data(), f64, 2, C, T2, W2, W2, 5, nullptr, 2, o2.data(), 1) == 1);
}

static double auc_bruteforce(const std::vector<double>& s, const std::vector<long>& y) {
  double num = 0, den = 0;
  for (size_t i = 0; i < s.size(); ++i)
    for (size_t j = 0; j < s.size(); ++j)
      if (y[i] == 1 && y[j] != 1) {
        den += 1;
        num += s[i] > s[j] ? 1.0 : (s[i] == s[j] ? 0.5 : 0.0);
      }
  return den > 0 ? num / den : 0.5;
}

static void check_metrics() {
  std::vector<double> s;
  std::vector<long> y;
  unsigned st = 12345u;
  for (int i = 0; i < 997; ++i) {
    st = st * 1664525u + 1013904223u;
    s.push_back((double)((st >> 8) % 37) / 37.0);  // heavy ties
    y.push_back((st >> 3) & 1);
  }
  CHECK(std::fabs(dnh_roc_auc(s.data(), y.data(), (long)s.size()) - auc_bruteforce(s, y)) < 1e-12);
  std::vector<long> ones(10, 1);
  CHECK(dnh_roc_auc(s.data(), ones.data(), 10) == 0.5);  // one class absent
  CHECK(dnh_roc_auc(s.data(), y.data(), 0) == 0.5);
  long cm[4];
  std::vector<long> pred(y.size());
  for (size_t i = 0; i < y.size(); ++i) pred[i] = s[i] > 0.5;
  CHECK(dnh_confusion2(pred.data(), y.data(), (long)y.size(), cm) == 0);
  long ref[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < y.size(); ++i) ref[(y[i] != 0) * 2 + (pred[i] != 0)]++;
  for (int k = 0; k < 4; ++k) CHECK(cm[k] == ref[k]);
  CHECK(cm[0] + cm[1] + cm[2] + cm[3] == (long)y.size());
  CHECK(dnh_confusion2(pred.data(), y.data(), 3, nullptr) == 1);
  CHECK(dnh_version() == 1);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <scratch dir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  check_fs(dir);
  check_windows_t<float>(0);
  check_windows_t<double>(1);
  check_metrics();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host sanitizer checks passed\n");
  return 0;
}
