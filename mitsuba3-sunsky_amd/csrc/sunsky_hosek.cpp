// sunsky_hosek.cpp -- the Hosek-Wilkie solar radiance of the reference's
// Python binding mi.hosek_sun_rad (src/render/python/sunsky_v.cpp:19), i.e.
// arhosekskymodel_solar_radiance_internal2 (ArHosekSkyModel.c:686-784) with
// arhosekskymodel_sr_internal (:655-684), restated in fp64 over the dataset
// tables: sun_spec_rad (turbidity, segment, lambda, control point; control
// points stored in ascending power order, sunsky.h:845-876) and sun_spec_ld.
#include <cmath>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "sunsky_dataset.h"
#include "sunsky_types.h"

namespace sunsky {

namespace {

struct SolarTables { std::vector<double> sun, ld; };

std::mutex g_mutex;
std::map<std::string, SolarTables> g_cache;

bool is_directory(const std::string& p);

const SolarTables& solar_tables(const std::string& where) {
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_cache.find(where);
    if (it != g_cache.end()) return it->second;
    Table sun, ld;
    std::string err;
    bool ok;
    if (is_directory(where)) {
        ok = read_array_file(where + "/sun_spec_rad.bin", 2, &sun, &err) &&
             read_array_file(where + "/sun_spec_ld.bin", 2, &ld, &err);
    } else {
        DatasetPack pack;
        ok = pack.open(where, &err) && pack.get("sun_spec_rad", &sun, &err) && pack.get("sun_spec_ld", &ld, &err);
    }
    if (!ok) throw std::runtime_error(err);
    if (sun.size() != (size_t)kNbTurbidity * kNbSunSegments * kNbWavelengths * kNbSunCtrlPts ||
        ld.size() != (size_t)kNbWavelengths * kNbSunLdParams)
        throw std::runtime_error("solar dataset has an unexpected size");
    SolarTables t{std::move(sun.data), std::move(ld.data)};
    return g_cache.emplace(where, std::move(t)).first->second;
}

}  // namespace

double hosek_solar_radiance(const std::string& datasets, double turbidity, double wavelength, double elevation,
                            double gamma) {
    if (!(wavelength >= 320.0 && wavelength <= 720.0 && turbidity >= 1.0 && turbidity <= 10.0)) return 0.0;
    const SolarTables& T = solar_tables(datasets);
    int turb_low = (int)turbidity - 1;
    double turb_frac = turbidity - (double)(turb_low + 1);
    if (turb_low == 9) { turb_low = 8; turb_frac = 1.0; }
    int wl_low = (int)((wavelength - 320.0) / 40.0);
    double wl_frac = std::fmod(wavelength, 40.0) / 40.0;
    if (wl_low == 10) { wl_low = 9; wl_frac = 1.0; }

    // arhosekskymodel_sr_internal: piecewise cubic in the elevation, 45 segments
    auto segment_radiance = [&](int turb, int wl) {
        int pos = (int)(std::pow(2.0 * elevation / 3.14159265358979323846, 1.0 / 3.0) * kNbSunSegments);
        if (pos > kNbSunSegments - 1) pos = kNbSunSegments - 1;
        const double break_x = std::pow((double)pos / (double)kNbSunSegments, 3.0) * (3.14159265358979323846 * 0.5);
        const double* c = &T.sun[(((size_t)turb * kNbSunSegments + pos) * kNbWavelengths + wl) * kNbSunCtrlPts];
        const double x = elevation - break_x;
        double res = 0.0, x_exp = 1.0;
        for (int i = 0; i < kNbSunCtrlPts; ++i) {
            res += x_exp * c[i];
            x_exp *= x;
        }
        return res;
    };
    double direct = (1.0 - turb_frac) * ((1.0 - wl_frac) * segment_radiance(turb_low, wl_low) +
                                         wl_frac * segment_radiance(turb_low, wl_low + 1)) +
                    turb_frac * ((1.0 - wl_frac) * segment_radiance(turb_low + 1, wl_low) +
                                 wl_frac * segment_radiance(turb_low + 1, wl_low + 1));
    double ld[kNbSunLdParams];
    for (int i = 0; i < kNbSunLdParams; ++i)
        ld[i] = (1.0 - wl_frac) * T.ld[wl_low * kNbSunLdParams + i] + wl_frac * T.ld[(wl_low + 1) * kNbSunLdParams + i];
    // sun distance to diameter ratio, squared (aperture 0.5358 deg)
    const double sol_rad_sin = std::sin(0.5358 / 2.0 * (3.14159265358979323846 / 180.0));
    const double ar2 = 1.0 / (sol_rad_sin * sol_rad_sin);
    const double singamma = std::sin(gamma);
    double sc2 = 1.0 - ar2 * singamma * singamma;
    if (sc2 < 0.0) sc2 = 0.0;
    const double sc = std::sqrt(sc2);
    const double dark = ld[0] + ld[1] * sc + ld[2] * std::pow(sc, 2.0) + ld[3] * std::pow(sc, 3.0) +
                        ld[4] * std::pow(sc, 4.0) + ld[5] * std::pow(sc, 5.0);
    return direct * dark;
}

namespace {
bool is_directory(const std::string& p) {
    std::vector<std::string> probe;
    FILE* f = std::fopen((p + "/sun_spec_rad.bin").c_str(), "rb");
    if (!f) return false;
    std::fclose(f);
    return true;
}
}  // namespace

}  // namespace sunsky
