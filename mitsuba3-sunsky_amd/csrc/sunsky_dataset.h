// sunsky_dataset.h -- dataset I/O for the sun/sky tables.
//
//  * DatasetPack: the product's own packed container (data/sunsky_datasets.pack,
//    written by tools/pack_datasets.py) holding the eight Hosek-Wilkie tables
//    plus the CIE-Y values the sampling-weight estimate needs.
//  * read_array_file / write_array_file: the reference's per-table ".bin"
//    format (array_from_file / array_to_file, sunsky.h:516-597) so a user can
//    point the emitter at an existing resources/sunsky/datasets directory.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace sunsky {

struct Table {
    std::vector<double> data;     // payload widened to fp64 (exact for fp32 files)
    std::vector<size_t> shape;
    int file_dtype = 0;           // 1 = fp32 on disk, 2 = fp64 on disk
    size_t size() const { return data.size(); }
};

class DatasetPack {
public:
    bool open(const std::string& path, std::string* err);
    bool get(const std::string& name, Table* out, std::string* err) const;
    const std::string& path() const { return path_; }
private:
    std::string path_;
    std::vector<unsigned char> buf_;
    uint32_t n_entries_ = 0;
};

// array_from_file (sunsky.h:516-561).  FileType is inferred from the payload
// size when file_dtype == 0, else forced (1 = float32, 2 = float64).
bool read_array_file(const std::string& path, int file_dtype, Table* out, std::string* err);
// array_to_file (sunsky.h:573-597): "SKY" magic, version 0, shape, fp32 payload.
bool write_array_file(const std::string& path, const float* data, size_t count,
                      const size_t* shape, int ndims, std::string* err);

uint32_t crc32_bytes(const unsigned char* p, size_t n);

}  // namespace sunsky
