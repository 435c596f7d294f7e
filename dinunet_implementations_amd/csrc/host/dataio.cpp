// Host-side runtime pieces in C++ (libdinunet_host.so, plain C ABI, OpenMP):
//
//  * FreeSurfer aseg-stats ingestion: every subject file of a site parsed in parallel and
//    max-normalised per subject into one fp32 matrix (reference comps/fs/__init__.py:33-39
//    re-parses one CSV per sample per epoch through pandas).
//  * ICA windowing with the reference semantics (S = T / W windows at offset j * stride, quirk
//    A9; comps/icalstm/__init__.py:26-34) for a selected subject list, straight into the
//    [n][S][C][W] fp32 layout the encoder GEMM reads, from fp32 or fp64 sources.
//  * Exact ROC-AUC (Mann-Whitney U with average ranks for ties) and a binary confusion matrix
//    over merged site predictions (the remote's global metrics).
//
// All entry points return 0 on success, a positive code on failure (documented per function).
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#define DNH_API extern "C" __attribute__((visibility("default")))

namespace {

// Parse one stats file: skip the header line, then "<name>\t<value>" (or whitespace separated)
// lines; the value is the LAST field.  Returns the number of values read (<= cap), or -1 when
// the file cannot be opened, -2 on a malformed value.
int parse_stats(const char* path, double* vals, int cap) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return -1;
  std::vector<char> buf;
  {
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) n = 0;
    buf.resize((size_t)n + 1);
    const size_t got = std::fread(buf.data(), 1, (size_t)n, f);
    buf[got] = '\0';
  }
  std::fclose(f);
  char* p = buf.data();
  // header
  while (*p && *p != '\n') ++p;
  if (*p == '\n') ++p;
  int count = 0;
  while (*p) {
    char* line = p;
    while (*p && *p != '\n') ++p;
    char* end = p;
    if (*p == '\n') ++p;
    while (end > line && (end[-1] == '\r' || end[-1] == ' ' || end[-1] == '\t')) --end;
    if (end == line) continue;  // blank line
    char* last = end;
    while (last > line && last[-1] != '\t' && last[-1] != ' ') --last;
    const char saved = *end;
    *end = '\0';
    errno = 0;
    char* stop = nullptr;
    const double v = std::strtod(last, &stop);
    *end = saved;
    if (stop == last || errno == ERANGE) return -2;
    if (count < cap) vals[count] = v;
    ++count;
  }
  return count < cap ? count : cap;
}

}  // namespace

// Parse n FreeSurfer stats files into out[n][nfeat] (fp32), each row divided by its own maximum
// (computed in fp64 like the reference's float64 DataFrame).  Rows with fewer than nfeat values
// are an error.  Returns 0, or 1 + (index of the first failing file) * 4 + kind with kind
// 1 = unreadable, 2 = malformed value, 3 = too few values.
DNH_API long dnh_fs_load(const char* const* paths, long n, int nfeat, float* out, int threads) {
  if (n <= 0) return 0;
  if (nfeat <= 0 || !out) return 1;
  long first_err = -1;
  int err_kind = 0;
#ifdef _OPENMP
  const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for num_threads(nt) schedule(dynamic, 8)
#endif
  for (long i = 0; i < n; ++i) {
    std::vector<double> vals((size_t)nfeat);
    const int got = parse_stats(paths[i], vals.data(), nfeat);
    int kind = 0;
    if (got == -1) kind = 1;
    else if (got == -2) kind = 2;
    else if (got < nfeat) kind = 3;
    if (kind) {
#ifdef _OPENMP
#pragma omp critical
#endif
      {
        if (first_err < 0 || i < first_err) { first_err = i; err_kind = kind; }
      }
      continue;
    }
    double mx = vals[0];
    for (int k = 1; k < nfeat; ++k) mx = std::max(mx, vals[k]);
    for (int k = 0; k < nfeat; ++k) out[i * (long)nfeat + k] = (float)(vals[k] / mx);
  }
  return first_err < 0 ? 0 : 1 + first_err * 4 + err_kind;
}

// Windows of the selected subjects: src[N][C][T] (fp32 when src_f64 == 0, else fp64) ->
// out[nrows][S][C][W] with out[i][j][c][w] = src[rows[i]][c][j * stride + w], S = T_used / W.
// Returns 0, 1 on bad arguments, 2 when a window runs past T or a row index is out of range.
DNH_API int dnh_ica_windows(const void* src, int src_f64, long N, int C, int T, int W, int stride,
                            int temporal, const long* rows, long nrows, float* out, int threads) {
  if (!src || !out || N < 0 || C <= 0 || T <= 0 || W <= 0 || stride <= 0 || temporal <= 0) return 1;
  const int S = temporal / W;
  if (S <= 0) return 1;
  if ((long)(S - 1) * stride + W > T) return 2;
  for (long i = 0; i < nrows; ++i)
    if ((rows ? rows[i] : i) < 0 || (rows ? rows[i] : i) >= N) return 2;
  const long per = (long)S * C * W;
#ifdef _OPENMP
  const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for collapse(2) num_threads(nt) schedule(static)
#endif
  for (long i = 0; i < nrows; ++i) {
    for (int j = 0; j < S; ++j) {
      const long r = rows ? rows[i] : i;
      float* o = out + i * per + (long)j * C * W;
      for (int c = 0; c < C; ++c) {
        const long base = (r * C + c) * (long)T + (long)j * stride;
        if (src_f64) {
          const double* s = static_cast<const double*>(src) + base;
          for (int w = 0; w < W; ++w) o[c * W + w] = (float)s[w];
        } else {
          const float* s = static_cast<const float*>(src) + base;
          std::memcpy(o + c * W, s, sizeof(float) * (size_t)W);
        }
      }
    }
  }
  return 0;
}

// Exact ROC-AUC of scores vs binary labels (label 1 = positive): Mann-Whitney U with average
// ranks over tied scores.  0.5 when a class is absent (as the Python metric).
DNH_API double dnh_roc_auc(const double* scores, const long* labels, long n) {
  if (n <= 0) return 0.5;
  long npos = 0;
  for (long i = 0; i < n; ++i) npos += labels[i] == 1;
  const long nneg = n - npos;
  if (npos == 0 || nneg == 0) return 0.5;
  std::vector<long> order((size_t)n);
  std::iota(order.begin(), order.end(), 0L);
  std::stable_sort(order.begin(), order.end(),
                   [&](long a, long b) { return scores[a] < scores[b]; });
  double rank_sum_pos = 0.0;
  long i = 0;
  while (i < n) {
    long j = i;
    while (j + 1 < n && scores[order[j + 1]] == scores[order[i]]) ++j;
    const double r = 0.5 * (double)(i + j) + 1.0;
    for (long k = i; k <= j; ++k)
      if (labels[order[k]] == 1) rank_sum_pos += r;
    i = j + 1;
  }
  return (rank_sum_pos - (double)npos * (double)(npos + 1) / 2.0) / ((double)npos * (double)nneg);
}

// Binary confusion counts of hard predictions: out = {tn, fp, fn, tp}.
DNH_API int dnh_confusion2(const long* pred, const long* labels, long n, long* out) {
  if (!out) return 1;
  out[0] = out[1] = out[2] = out[3] = 0;
  for (long i = 0; i < n; ++i) {
    const int p = pred[i] != 0, y = labels[i] != 0;
    out[(y << 1) | p] += 1;
  }
  return 0;
}

DNH_API int dnh_version() { return 1; }
