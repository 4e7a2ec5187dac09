// sunsky_dataset.cpp -- see sunsky_dataset.h.
#include "sunsky_dataset.h"

#include <cstdio>
#include <cstring>

namespace sunsky {

namespace {
constexpr size_t kEntrySize = 96;

bool read_all(const std::string& path, std::vector<unsigned char>* buf, std::string* err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        *err = "\"" + path + "\": file does not exist!";   // sunsky.h:519-520
        return false;
    }
    std::fseek(f, 0, SEEK_END);
    long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf->resize(sz > 0 ? (size_t)sz : 0);
    bool ok = sz >= 0 && std::fread(buf->data(), 1, buf->size(), f) == buf->size();
    std::fclose(f);
    if (!ok) *err = "\"" + path + "\": read error";
    return ok;
}

template <typename T> T load_le(const unsigned char* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }
}  // namespace

uint32_t crc32_bytes(const unsigned char* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

bool DatasetPack::open(const std::string& path, std::string* err) {
    path_ = path;
    if (!read_all(path, &buf_, err)) return false;
    if (buf_.size() < 16 || std::memcmp(buf_.data(), "SSKYPAK1", 8) != 0) {
        *err = "\"" + path + "\": not a sunsky dataset pack";
        return false;
    }
    uint32_t version = load_le<uint32_t>(&buf_[8]);
    n_entries_ = load_le<uint32_t>(&buf_[12]);
    if (version != 1 || 16 + n_entries_ * kEntrySize > buf_.size()) {
        *err = "\"" + path + "\": unsupported pack version";
        return false;
    }
    return true;
}

bool DatasetPack::get(const std::string& name, Table* out, std::string* err) const {
    for (uint32_t i = 0; i < n_entries_; ++i) {
        const unsigned char* e = &buf_[16 + i * kEntrySize];
        if (std::strncmp((const char*)e, name.c_str(), 24) != 0) continue;
        uint32_t dtype = load_le<uint32_t>(e + 24), ndims = load_le<uint32_t>(e + 28);
        uint64_t off = load_le<uint64_t>(e + 80);
        uint32_t nbytes = load_le<uint32_t>(e + 88), crc = load_le<uint32_t>(e + 92);
        if (ndims > 6 || (dtype != 1 && dtype != 2) || off + nbytes > buf_.size()) break;
        out->shape.clear();
        size_t count = 1;
        for (uint32_t d = 0; d < ndims; ++d) {
            size_t s = (size_t)load_le<uint64_t>(e + 32 + 8 * d);
            out->shape.push_back(s);
            count *= s;
        }
        size_t esz = dtype == 2 ? 8 : 4;
        if (count * esz != nbytes) break;
        if (crc32_bytes(&buf_[off], nbytes) != crc) {
            *err = "dataset pack entry '" + name + "' failed its CRC check";
            return false;
        }
        out->file_dtype = (int)dtype;
        out->data.resize(count);
        for (size_t k = 0; k < count; ++k)
            out->data[k] = dtype == 2 ? load_le<double>(&buf_[off + 8 * k])
                                      : (double)load_le<float>(&buf_[off + 4 * k]);
        return true;
    }
    *err = "dataset pack \"" + path_ + "\" has no (valid) entry '" + name + "'";
    return false;
}

bool read_array_file(const std::string& path, int file_dtype, Table* out, std::string* err) {
    std::vector<unsigned char> buf;
    if (!read_all(path, &buf, err)) return false;
    // Header: char[3] magic, uint32 version, uint64 ndims, uint64 shape[ndims]
    if (buf.size() < 15 || (std::memcmp(buf.data(), "SKY", 3) != 0 && std::memcmp(buf.data(), "SUN", 3) != 0)) {
        *err = "OUPSSS wrong file";   // the reference's message, sunsky.h:531-532
        return false;
    }
    uint64_t ndims = load_le<uint64_t>(&buf[7]);
    if (ndims > 16 || 15 + 8 * ndims > buf.size()) {
        *err = "\"" + path + "\": corrupt header";
        return false;
    }
    out->shape.clear();
    size_t count = 1;
    for (uint64_t d = 0; d < ndims; ++d) {
        size_t s = (size_t)load_le<uint64_t>(&buf[15 + 8 * d]);
        if (!s) {
            *err = "Got dimension with 0 elements";   // sunsky.h:547-548
            return false;
        }
        out->shape.push_back(s);
        count *= s;
    }
    size_t off = 15 + 8 * ndims, payload = buf.size() - off;
    if (file_dtype == 0) file_dtype = payload == 8 * count ? 2 : (payload == 4 * count ? 1 : 0);
    size_t esz = file_dtype == 2 ? 8 : 4;
    if (file_dtype == 0 || payload < count * esz) {
        *err = "\"" + path + "\": payload does not match its shape";
        return false;
    }
    out->file_dtype = file_dtype;
    out->data.resize(count);
    for (size_t k = 0; k < count; ++k)
        out->data[k] = file_dtype == 2 ? load_le<double>(&buf[off + 8 * k]) : (double)load_le<float>(&buf[off + 4 * k]);
    return true;
}

bool write_array_file(const std::string& path, const float* data, size_t count, const size_t* shape,
                      int ndims, std::string* err) {
    std::vector<size_t> sh(shape, shape + (ndims > 0 ? ndims : 0));
    if (sh.empty()) sh.push_back(count);
    size_t prod = 1;
    for (size_t s : sh) {
        if (!s) { *err = "Got dimension with 0 elements"; return false; }
        prod *= s;
    }
    if (prod != count) { *err = "shape does not match the element count"; return false; }
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { *err = "\"" + path + "\": cannot open for writing"; return false; }
    uint32_t version = 0;
    uint64_t nd = sh.size();
    bool ok = std::fwrite("SKY", 1, 3, f) == 3 && std::fwrite(&version, 4, 1, f) == 1 &&
              std::fwrite(&nd, 8, 1, f) == 1;
    for (size_t s : sh) { uint64_t v = s; ok = ok && std::fwrite(&v, 8, 1, f) == 1; }
    ok = ok && std::fwrite(data, sizeof(float), count, f) == count;
    std::fclose(f);
    if (!ok) *err = "\"" + path + "\": write error";
    return ok;
}

}  // namespace sunsky
