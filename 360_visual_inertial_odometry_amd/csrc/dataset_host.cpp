// dataset_host.cpp — the dataset formats on either side of the path: the camera
// timestamp list and the IMU CSV the demo app feeds the estimator with.
//
// Reference: LoadCameraTimestamps / LoadIMUData (app/main.cpp:30-90).  Same acceptance rules:
// timestamps — one value per line, empty lines skipped, a line without a leading number skipped
// (std::stod); IMU — the first line is a header and always skipped, then lines split on ',' must
// give exactly 7 fields t,ax,ay,az,gx,gy,gz (std::stod for t, std::stof for the rest), any field
// that does not convert (or overflows) drops the line.  Host code: no device work.
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "vio360.h"

namespace {

bool parse_double(const std::string& s, double* v) {
    try {
        *v = std::stod(s);
        return true;
    } catch (...) {
        return false;
    }
}

bool parse_float(const std::string& s, float* v) {
    try {
        *v = std::stof(s);
        return true;
    } catch (...) {
        return false;
    }
}

}  // namespace

extern "C" int vio_load_camera_timestamps(const char* path, double* out, int cap, int* n) {
    if (!path || !n || cap < 0 || (cap > 0 && !out)) return VIO_EINVAL;
    std::ifstream f(path);
    if (!f.is_open()) return VIO_EINVAL;
    int count = 0;
    std::string line;
    while (std::getline(f, line)) {
        double t;
        if (line.empty() || !parse_double(line, &t)) continue;
        if (count < cap) out[count] = t;
        ++count;
    }
    *n = count;
    return VIO_OK;
}

extern "C" int vio_load_imu_csv(const char* path, vio_imu_data* out, int cap, int* n) {
    if (!path || !n || cap < 0 || (cap > 0 && !out)) return VIO_EINVAL;
    std::ifstream f(path);
    if (!f.is_open()) return VIO_EINVAL;
    int count = 0;
    std::string line;
    std::getline(f, line);  // header
    std::vector<std::string> fields;
    while (std::getline(f, line)) {
        if (line.empty()) continue;
        fields.clear();
        std::stringstream ss(line);
        std::string item;
        while (std::getline(ss, item, ',')) fields.push_back(item);
        if (fields.size() != 7) continue;
        vio_imu_data m;
        if (!parse_double(fields[0], &m.timestamp) || !parse_float(fields[1], &m.ax) ||
            !parse_float(fields[2], &m.ay) || !parse_float(fields[3], &m.az) || !parse_float(fields[4], &m.gx) ||
            !parse_float(fields[5], &m.gy) || !parse_float(fields[6], &m.gz))
            continue;
        if (count < cap) out[count] = m;
        ++count;
    }
    *n = count;
    return VIO_OK;
}
