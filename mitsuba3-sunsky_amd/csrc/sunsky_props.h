// sunsky_props.h -- a minimal property bag with the semantics the reference
// plugin relies on (mitsuba::Properties as used by init_from_props,
// sunsky.cpp:889-948): typed getters with defaults, has_property(), and the
// "unreferenced property" check the scene loader applies after construction
// (src/core/xml.cpp:1085-1102).
#pragma once
#include <cmath>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace sunsky {

class Properties {
public:
    enum class Type { Float, Int, Vector3, Transform, Spectrum, Irregular, String };

    struct Value {
        Type type = Type::Float;
        double f = 0;
        int64_t i = 0;
        float m[16] = {0};
        std::vector<float> a, b;   // Spectrum: a = values; Irregular: a = wavelengths, b = values
        std::string s;
        mutable bool queried = false;
    };

    void set_float(const std::string& k, double v) { Value x; x.type = Type::Float; x.f = v; map_[k] = x; }
    void set_int(const std::string& k, int64_t v) { Value x; x.type = Type::Int; x.i = v; map_[k] = x; }
    void set_vector3(const std::string& k, float a, float b, float c) {
        Value x; x.type = Type::Vector3; x.m[0] = a; x.m[1] = b; x.m[2] = c; map_[k] = x;
    }
    void set_transform(const std::string& k, const float* m16) {
        Value x; x.type = Type::Transform;
        for (int i = 0; i < 16; ++i) x.m[i] = m16[i];
        map_[k] = x;
    }
    void set_spectrum(const std::string& k, const float* v, int n) {
        Value x; x.type = Type::Spectrum; x.a.assign(v, v + n); map_[k] = x;
    }
    void set_irregular(const std::string& k, const float* wl, const float* v, int n) {
        Value x; x.type = Type::Irregular; x.a.assign(wl, wl + n); x.b.assign(v, v + n); map_[k] = x;
    }
    void set_string(const std::string& k, const std::string& v) { Value x; x.type = Type::String; x.s = v; map_[k] = x; }

    bool has(const std::string& k) const { return map_.count(k) != 0; }

    const Value* find(const std::string& k) const {
        auto it = map_.find(k);
        if (it == map_.end()) return nullptr;
        it->second.queried = true;
        return &it->second;
    }

    double get_float(const std::string& k, double def) const {
        const Value* v = find(k);
        if (!v) return def;
        if (v->type == Type::Float) return v->f;
        if (v->type == Type::Int) return (double)v->i;
        throw std::invalid_argument("Property \"" + k + "\" has the wrong type (expected float)");
    }

    int64_t get_int(const std::string& k, int64_t def) const {
        const Value* v = find(k);
        if (!v) return def;
        if (v->type == Type::Int) return v->i;
        if (v->type == Type::Float && std::floor(v->f) == v->f) return (int64_t)v->f;
        throw std::invalid_argument("Property \"" + k + "\" has the wrong type (expected integer)");
    }

    const Value* get_typed(const std::string& k, Type t) const {
        const Value* v = find(k);
        if (v && v->type != t)
            throw std::invalid_argument("Property \"" + k + "\" has the wrong type");
        return v;
    }

    std::vector<std::string> unqueried() const {
        std::vector<std::string> r;
        for (auto& kv : map_)
            if (!kv.second.queried && kv.first != "type" && kv.first != "id") r.push_back(kv.first);
        return r;
    }

private:
    std::map<std::string, Value> map_;
};

}  // namespace sunsky
