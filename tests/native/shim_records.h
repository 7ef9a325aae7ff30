// Named arrays written by tests/test_shims_gpu.py (write_records): per record a 48-byte NUL-padded
// name, an int64 byte count, then the raw little-endian bytes.  Test infrastructure for the
// *_shim_gpu checks.
#ifndef ORBGPU_TESTS_SHIM_RECORDS_H
#define ORBGPU_TESTS_SHIM_RECORDS_H

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

struct Records {
    std::map<std::string, std::vector<uint8_t>> rec;

    bool Load(const char* path) {
        FILE* f = std::fopen(path, "rb");
        if (!f) return false;
        for (;;) {
            char name[49] = {};
            if (std::fread(name, 1, 48, f) != 48) break;
            int64_t n = 0;
            if (std::fread(&n, 8, 1, f) != 1 || n < 0) break;
            std::vector<uint8_t> b((size_t)n);
            if (n && std::fread(b.data(), 1, (size_t)n, f) != (size_t)n) break;
            rec[name] = std::move(b);
        }
        std::fclose(f);
        return !rec.empty();
    }
    bool Has(const std::string& k) const { return rec.count(k) != 0; }
    template <class T>
    std::vector<T> Get(const std::string& k) const {
        auto it = rec.find(k);
        if (it == rec.end()) throw std::runtime_error("missing record " + k);
        std::vector<T> v(it->second.size() / sizeof(T));
        if (!v.empty()) std::memcpy(v.data(), it->second.data(), v.size() * sizeof(T));
        return v;
    }
    template <class T>
    T Scalar(const std::string& k) const {
        const auto v = Get<T>(k);
        if (v.size() != 1) throw std::runtime_error("record " + k + " is not a scalar");
        return v[0];
    }
};

#endif
