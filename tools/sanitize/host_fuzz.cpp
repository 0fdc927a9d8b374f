// host_fuzz — the host side of libpqgpu (Thrift footer/page-header parser, format.cpp; chunk
// planner, host.cpp) over untrusted bytes, built with AddressSanitizer + UBSan (tools/sanitize/
// Makefile). No GPU: a plan-only batch (ctx == NULL) walks and validates every page header,
// decompresses GZIP / dictionary pages and stages sections, exactly the code the decode path
// runs on the host before any upload.
//
// For every file argument: the file as is, then `mutations` seeded variants (byte flips, bytes
// set to 0x00 / 0xff / 0x80, truncations, a duplicated range), each opened and planned for every
// column chunk with and without CRC validation. The harness only has to finish: a sanitizer
// report aborts the process with a non-zero status.
//
// usage: host_fuzz [-m mutations] [-s seed] file...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pqgpu.h"

static std::vector<uint8_t> read_file(const char *path) {
  std::vector<uint8_t> v;
  FILE *f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

// Open and plan every chunk; returns the number of chunks planned without error.
static int plan(const std::vector<uint8_t> &d) {
  pqgpu_file *f = nullptr;
  pqgpu_error e;
  if (pqgpu_file_open(d.data(), d.size(), &f, &e) != 0) return 0;
  int ok = 0;
  const int nrg = pqgpu_file_num_row_groups(f), nc = pqgpu_file_num_columns(f);
  for (int crc = 0; crc < 2; crc++) {
    pqgpu_batch *b = nullptr;
    if (pqgpu_batch_create(nullptr, &b, &e) != 0) break;
    for (int rg = 0; rg < nrg; rg++)
      for (int c = 0; c < nc; c++) {
        int32_t id = -1;
        pqgpu_chunk_meta meta;
        (void)pqgpu_file_chunk_meta(f, rg, c, &meta, &e);
        if (pqgpu_batch_add_file_chunk(b, f, rg, c, crc, &id, &e) == 0) ok++;
      }
    pqgpu_batch_stats st;
    (void)pqgpu_batch_stats_get(b, &st);
    pqgpu_batch_destroy(b);
  }
  pqgpu_file_close(f);
  return ok;
}

static std::vector<uint8_t> mutate(const std::vector<uint8_t> &d, std::mt19937_64 &rng) {
  std::vector<uint8_t> m = d;
  if (m.empty()) return m;
  const int kind = (int)(rng() % 6);
  const size_t n = m.size();
  // bias positions toward the footer (the Thrift metadata) and the first page headers
  auto pos = [&]() -> size_t {
    const uint64_t r = rng();
    if (r % 3 == 0 && n > 64) return n - 1 - (size_t)((r >> 8) % std::min<size_t>(n, 4096));
    if (r % 3 == 1) return (size_t)((r >> 8) % std::min<size_t>(n, 4096));
    return (size_t)((r >> 8) % n);
  };
  switch (kind) {
    case 0: for (int k = 0; k < 1 + (int)(rng() % 4); k++) m[pos()] ^= (uint8_t)(1u << (rng() % 8)); break;
    case 1: m[pos()] = 0x00; break;
    case 2: m[pos()] = 0xff; break;
    case 3: m[pos()] = 0x80; break;
    case 4: m.resize(pos()); break;
    default: {
      const size_t a = pos(), len = std::min<size_t>(n - a, 1 + rng() % 64), at = pos();
      std::vector<uint8_t> piece(m.begin() + a, m.begin() + a + len);
      m.insert(m.begin() + at, piece.begin(), piece.end());
    }
  }
  return m;
}

int main(int argc, char **argv) {
  int mutations = 200;
  uint64_t seed = 1;
  std::vector<std::string> files;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "-m") && i + 1 < argc) mutations = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-s") && i + 1 < argc) seed = strtoull(argv[++i], nullptr, 10);
    else files.push_back(argv[i]);
  }
  long total = 0, planned = 0;
  for (const std::string &path : files) {
    const std::vector<uint8_t> d = read_file(path.c_str());
    std::mt19937_64 rng(seed ^ std::hash<std::string>{}(path));
    planned += plan(d);
    total++;
    for (int k = 0; k < mutations; k++) {
      planned += plan(mutate(d, rng));
      total++;
    }
  }
  printf("host_fuzz: %ld images, %ld chunks planned without error\n", total, planned);
  return 0;
}
