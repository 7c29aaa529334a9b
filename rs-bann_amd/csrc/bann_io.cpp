// bann_io.cpp — the files on either side of the path (host only): PLINK .bed
// dims, ExternalGrouping / UniformGrouping marker index lists and the bincode
// .phen phenotypes.  bann_genotypes_load_bed (device streaming) is in bann_io_dev.hip.
//
//   BedDims::from_dims_file / from_plink_fileset     io/dims.rs:15-34
//   ExternalGrouping::from_file                       group/external.rs:15-60
//   UniformGrouping::new                              group/uniform.rs:11-23
//   Phenotypes::from_file / to_file (bincode Vec<f32>) data/phenotypes.rs:28-36
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/bann.h"

static int64_t count_lines(const std::string& path) {
  std::ifstream f(path);
  if (!f) return -1;
  int64_t k = 0;
  std::string line;
  while (std::getline(f, line)) ++k;
  return k;
}

extern "C" int bann_bed_dims(const char* stem, int64_t* n_out, int64_t* num_markers_out) {
  if (!stem || !n_out || !num_markers_out) return BANN_E_ARG;
  const std::string s(stem);
  std::ifstream dims(s + ".dims");
  if (dims) {  // "num_individuals num_markers" on the first line
    int64_t n = -1, m = -1;
    std::string line;
    std::getline(dims, line);
    std::istringstream ls(line);
    if (!(ls >> n >> m) || n <= 0 || m <= 0) return BANN_E_SHAPE;
    *n_out = n;
    *num_markers_out = m;
    return BANN_OK;
  }
  const int64_t n = count_lines(s + ".fam"), m = count_lines(s + ".bim");  // one line per individual / marker
  if (n <= 0 || m <= 0) return BANN_E_ARG;
  *n_out = n;
  *num_markers_out = m;
  return BANN_OK;
}

// two-column text "marker_ix group_ix" (0-based); groups must be 0 .. G-1; markers
// keep their file order within a group.  CSR result: offsets[G+1], markers[entries].
extern "C" int bann_grouping_read(const char* path, int32_t* num_groups, int64_t* num_entries, int64_t* offsets,
                                  int32_t* markers) {
  if (!path || !num_groups || !num_entries) return BANN_E_ARG;
  std::ifstream f(path);
  if (!f) return BANN_E_ARG;
  std::map<int64_t, std::vector<int32_t>> groups;
  std::string line;
  int64_t entries = 0;
  while (std::getline(f, line)) {
    std::istringstream ls(line);
    int64_t mk, g;
    if (!(ls >> mk >> g)) {
      if (line.find_first_not_of(" \t\r") == std::string::npos) continue;  // blank line
      return BANN_E_SHAPE;
    }
    if (mk < 0 || g < 0 || mk > INT32_MAX) return BANN_E_SHAPE;
    groups[g].push_back((int32_t)mk);
    ++entries;
  }
  const int64_t G = (int64_t)groups.size();
  if (G > 0 && groups.rbegin()->first != G - 1) return BANN_E_SHAPE;  // continuous 0-based indices (external.rs:46-49)
  *num_groups = (int32_t)G;
  *num_entries = entries;
  if (offsets && markers) {
    int64_t o = 0;
    for (int64_t g = 0; g < G; ++g) {
      offsets[g] = o;
      for (int32_t mk : groups[g]) markers[o++] = mk;
    }
    offsets[G] = o;
  }
  return BANN_OK;
}

extern "C" int bann_grouping_uniform(int32_t num_groups, int32_t group_size, int64_t* offsets, int32_t* markers) {
  if (num_groups <= 0 || group_size <= 0 || !offsets || !markers) return BANN_E_ARG;
  for (int64_t g = 0; g <= num_groups; ++g) offsets[g] = g * group_size;
  for (int64_t i = 0; i < (int64_t)num_groups * group_size; ++i) markers[i] = (int32_t)i;
  return BANN_OK;
}

// bincode 1.3 (legacy config) of `struct Phenotypes { y: Vec<f32> }`: u64 length, then the values, little endian
extern "C" int bann_phen_read(const char* path, int64_t* n_out, float* y_out) {
  if (!path || !n_out) return BANN_E_ARG;
  FILE* f = fopen(path, "rb");
  if (!f) return BANN_E_ARG;
  uint64_t len = 0;
  int rc = BANN_OK;
  if (fread(&len, 8, 1, f) != 1) {
    rc = BANN_E_SHAPE;
  } else {
    *n_out = (int64_t)len;
    if (y_out && fread(y_out, sizeof(float), len, f) != len) rc = BANN_E_SHAPE;
  }
  fclose(f);
  return rc;
}

extern "C" int bann_phen_write(const char* path, const float* y, int64_t n) {
  if (!path || !y || n < 0) return BANN_E_ARG;
  FILE* f = fopen(path, "wb");
  if (!f) return BANN_E_ARG;
  const uint64_t len = (uint64_t)n;
  const bool ok = fwrite(&len, 8, 1, f) == 1 && fwrite(y, sizeof(float), (size_t)n, f) == (size_t)n;
  return (fclose(f) == 0 && ok) ? BANN_OK : BANN_E_ARG;
}
