// Matching-file reader: the reference's get_data
// (Phase 1/Utils.py:8-64) builds three dense n_features x n_images
// matrices with a Python loop per line; at cfg5 scale those are 800 MB
// each.  Here the files are parsed natively into a COO observation store
// (feature, image, x, y), which the dense view and the BA observation lists
// are both built from.
//
// Semantics kept from the reference, per line of matching<n>.txt
// (n = 1 .. no_of_images-1, first line skipped):
//   tokens = line.split(); cols = [float(t) for t in tokens]
//   image n gets (cols[4], cols[5]) as floats;
//   while cols[0] > 1 (decremented): image int(cols[5+m]) gets
//   (int(cols[6+m]), int(cols[7+m])) -- truncated toward zero; later writes
//   to the same image win; image_id - 1 < 0 wraps like a Python index.
// Decimal -> double uses std::from_chars (correctly rounded, like float()).
// Files are read whole and split into newline-aligned chunks parsed by a
// thread pool; rows keep file order (feature index = line ordinal).
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host_pool.hpp"
#include "sfm_common.hpp"

namespace {

struct Obs {
    int32_t img;
    double x, y;
};

struct Chunk {
    std::vector<int32_t> row_len;  // observations per row
    std::vector<Obs> obs;
    std::string error;
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

bool parse_double(const char *&p, const char *end, double &v) {
    while (p < end && is_space(*p)) ++p;
    if (p >= end) return false;
    const char *q = p;
    if (*q == '+') ++q;  // float() accepts a leading '+', from_chars does not
    auto r = std::from_chars(q, end, v);
    if (r.ec != std::errc() || (r.ptr < end && !is_space(*r.ptr))) return false;
    p = r.ptr;
    return true;
}

// Python int(float): truncation toward zero, error for nan / inf
bool py_int(double v, double &out) {
    if (!std::isfinite(v)) return false;
    out = std::trunc(v);
    return true;
}

void parse_range(const char *b, const char *e, int file_image, int n_img, Chunk &out) {
    const char *p = b;
    std::vector<double> cols;
    std::vector<Obs> row;
    while (p < e) {
        const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(e - p)));
        const char *le = nl ? nl : e;
        cols.clear();
        const char *q = p;
        for (;;) {
            while (q < le && is_space(*q)) ++q;
            if (q >= le) break;
            double v;
            if (!parse_double(q, le, v)) {
                out.error = "could not convert string to float: '" +
                            std::string(q, (size_t)std::min<ptrdiff_t>(le - q, 32)) + "'";
                return;
            }
            cols.push_back(v);
        }
        if (cols.size() < 6) {
            out.error = "index out of range: a row needs at least 6 columns";
            return;
        }
        row.clear();
        row.push_back({file_image - 1, cols[4], cols[5]});
        double nm = cols[0];
        size_t m = 1;
        while (nm > 1) {
            if (7 + m >= cols.size()) {
                out.error = "index out of range: match triple past the end of the row";
                return;
            }
            double id, xi, yi;
            if (!py_int(cols[5 + m], id) || !py_int(cols[6 + m], xi) || !py_int(cols[7 + m], yi)) {
                out.error = "cannot convert float NaN or infinity to integer";
                return;
            }
            m += 3;
            nm = nm - 1;
            int64_t k = (int64_t)id - 1;
            if (k < 0) k += n_img;
            if (k < 0 || k >= n_img) {
                out.error = "index " + std::to_string((int64_t)id - 1) + " is out of bounds for axis 1";
                return;
            }
            row.push_back({(int32_t)k, xi, yi});
        }
        // last write to an image wins; emit image-ascending
        std::stable_sort(row.begin(), row.end(), [](const Obs &a, const Obs &c) { return a.img < c.img; });
        int32_t kept = 0;
        for (size_t i = 0; i < row.size(); ++i) {
            if (i + 1 < row.size() && row[i + 1].img == row[i].img) continue;
            out.obs.push_back(row[i]);
            ++kept;
        }
        out.row_len.push_back(kept);
        p = nl ? nl + 1 : e;
    }
}

struct Store {
    int64_t n_features = 0;
    std::vector<int32_t> feature, image;
    std::vector<double> x, y;
};

}  // namespace

using namespace sfm;

extern "C" int sfm_matching_parse(const char *data_path, int32_t no_of_images, int32_t n_threads, void **handle,
                                  int64_t *n_features, int64_t *n_obs) {
    SFM_CHECK_ARG(data_path && handle && n_features && n_obs, "null pointer");
    SFM_CHECK_ARG(no_of_images >= 1, "no_of_images must be >= 1");
    *handle = nullptr;
    auto st = new Store();
    const int nt = n_threads > 0 ? n_threads : host_threads();
    for (int n = 1; n < no_of_images; ++n) {
        const std::string path = std::string(data_path) + "/matching" + std::to_string(n) + ".txt";
        FILE *f = std::fopen(path.c_str(), "rb");
        if (!f) {
            delete st;
            set_error("No such file or directory: '%s'", path.c_str());
            return SFM_ERR_ARG;
        }
        std::vector<char> buf;
        char tmp[1 << 16];
        size_t r;
        while ((r = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
        std::fclose(f);
        const char *b = buf.data(), *e = b + buf.size();
        const char *first = static_cast<const char *>(memchr(b, '\n', buf.size()));
        b = first ? first + 1 : e;  // skip the header line
        // newline-aligned chunks, >= 256 KiB each
        const size_t len = (size_t)(e - b);
        const int nchunks = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, len / (256 << 10)));
        std::vector<const char *> cut(nchunks + 1, e);
        cut[0] = b;
        for (int k = 1; k < nchunks; ++k) {
            const char *c = b + len * k / nchunks;
            if (c < cut[k - 1]) c = cut[k - 1];
            const char *nl = static_cast<const char *>(memchr(c, '\n', (size_t)(e - c)));
            cut[k] = nl ? nl + 1 : e;
        }
        std::vector<Chunk> chunks(nchunks);
        std::vector<std::thread> pool;
        for (int k = 1; k < nchunks; ++k)
            pool.emplace_back(parse_range, cut[k], cut[k + 1], n, (int)no_of_images, std::ref(chunks[k]));
        parse_range(cut[0], cut[1], n, no_of_images, chunks[0]);
        for (auto &t : pool) t.join();
        for (int k = 0; k < nchunks; ++k) {
            if (!chunks[k].error.empty()) {
                delete st;
                set_error("%s: %s", path.c_str(), chunks[k].error.c_str());
                return SFM_ERR_ARG;
            }
            size_t o = 0;
            for (int32_t rl : chunks[k].row_len) {
                for (int32_t j = 0; j < rl; ++j, ++o) {
                    const Obs &ob = chunks[k].obs[o];
                    st->feature.push_back((int32_t)st->n_features);
                    st->image.push_back(ob.img);
                    st->x.push_back(ob.x);
                    st->y.push_back(ob.y);
                }
                ++st->n_features;
            }
        }
    }
    *handle = st;
    *n_features = st->n_features;
    *n_obs = (int64_t)st->feature.size();
    return 0;
}

extern "C" int sfm_matching_read(void *handle, int32_t *feature, int32_t *image, double *x, double *y) {
    SFM_CHECK_ARG(handle, "null handle");
    auto st = static_cast<Store *>(handle);
    const size_t n = st->feature.size();
    if (n) {
        SFM_CHECK_ARG(feature && image && x && y, "null pointer");
        std::memcpy(feature, st->feature.data(), n * sizeof(int32_t));
        std::memcpy(image, st->image.data(), n * sizeof(int32_t));
        std::memcpy(x, st->x.data(), n * sizeof(double));
        std::memcpy(y, st->y.data(), n * sizeof(double));
    }
    return 0;
}

extern "C" int sfm_matching_free(void *handle) {
    delete static_cast<Store *>(handle);
    return 0;
}
