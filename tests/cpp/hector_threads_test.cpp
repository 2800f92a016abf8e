// tests/cpp/hector_threads_test.cpp -- TEST INFRASTRUCTURE.  The MapRepHip drop-in's threading contract,
// exercised through slam2d::HectorMapBackend (include/slam2d/hector_map_backend.hpp) and the C-ABI:
//
//   spin thread    : HectorSlamProcessor::update for every scan (hs_update; hector_slam.cc:201)
//   publish thread : getGridMap(0) in a loop (hs_get_map; hector_slam.cc:254-317), recording every
//                    refreshed mirror's (update index, hash of every cell's log-odds bits + updateIndex)
//
// and checked against the CPU oracle (oracle/build/libhector_oracle.so, the kernels' reduction order):
// every snapshot the publish thread saw equals the oracle's map after the same number of updates, the
// update index only moves forward and moved while the spin thread ran, and every pose is bit-exact.
//
// usage: hector_threads_test <scans.bin> <map_size> <levels>
//   scans.bin: int32 K, int32 max_points, int32 counts[K], float32 points[K][max_points][2] (map scale)
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <thread>
#include <vector>

#include <slam2d/hector_map_backend.hpp>

extern "C" {  // oracle/hector_oracle.c
struct ho_ctx;
ho_ctx *ho_create(float map_resolution, int map_size_x, int map_size_y, float start_x, float start_y, int levels);
void ho_destroy(ho_ctx *c);
void ho_set_update_factors(ho_ctx *c, float free_factor, float occ_factor);
void ho_set_thresholds(ho_ctx *c, float min_dist, float min_ang);
void ho_set_mode(ho_ctx *c, int reduce_threads, int use_libm);
int ho_process(ho_ctx *c, const float *xy, int n, float ox, float oy, const float *hint, int map_without_matching,
               float *pose_out, float *cov_out);
void ho_get_last_pose(const ho_ctx *c, float *pose);
void ho_get_level(const ho_ctx *c, int lvl, float *l_out, int *upd_out);
int ho_update_index(const ho_ctx *c, int lvl);
}

static uint64_t fnv(const void *p, size_t n, uint64_t h = 1469598103934665603ull)
{
    const unsigned char *b = static_cast<const unsigned char *>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s scans.bin map_size levels\n", argv[0]);
        return 2;
    }
    const int size = atoi(argv[2]), levels = atoi(argv[3]);
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t K = 0, M = 0;
    if (fread(&K, 4, 1, f) != 1 || fread(&M, 4, 1, f) != 1) return 2;
    std::vector<int32_t> counts(K);
    std::vector<float> pts((size_t)K * M * 2);
    if (fread(counts.data(), 4, K, f) != (size_t)K || fread(pts.data(), 4, pts.size(), f) != pts.size()) return 2;
    fclose(f);
    const size_t cells = (size_t)size * size;

    // ---- oracle: the map after every update (forced updates: update index k after scan k)
    std::map<int, uint64_t> want;
    std::vector<float> opose((size_t)K * 3);
    {
        ho_ctx *o = ho_create(0.05f, size, size, 0.5f, 0.5f, levels);
        ho_set_mode(o, 0, 0);  // the reference summation order: the library default
        ho_set_update_factors(o, 0.4f, 0.9f);
        ho_set_thresholds(o, -1.0f, -1.0f);
        std::vector<float> l(cells);
        std::vector<int> u(cells);
        ho_get_level(o, 0, l.data(), u.data());
        want[ho_update_index(o, 0)] = fnv(u.data(), 4 * cells, fnv(l.data(), 4 * cells));
        for (int k = 0; k < K; ++k) {
            float hint[3], cov[9];
            ho_get_last_pose(o, hint);
            ho_process(o, &pts[(size_t)k * M * 2], counts[k], 0.0f, 0.0f, hint, 0, &opose[3 * k], cov);
            ho_get_level(o, 0, l.data(), u.data());
            want[ho_update_index(o, 0)] = fnv(u.data(), 4 * cells, fnv(l.data(), 4 * cells));
        }
        ho_destroy(o);
    }

    // ---- device: spin thread updates, publish thread refreshes
    slam2d::HectorMapBackend be(0.05f, size, size, levels, 0.5f, 0.5f, M);
    be.setUpdateFactorFree(0.4f);
    be.setUpdateFactorOccupied(0.9f);
    be.setMapUpdateThresholds(-1.0f, -1.0f);
    std::atomic<bool> done{false};
    std::vector<float> gpose((size_t)K * 3);
    std::vector<std::pair<int, uint64_t>> seen;
    int errors = 0;
    std::thread spin([&] {
        for (int k = 0; k < K; ++k) {
            float cov[9];
            be.process(&pts[(size_t)k * M * 2], counts[k], 0.0f, 0.0f, nullptr, false, &gpose[3 * k], cov);
            // the sensor period (a 40 Hz laser leaves 25 ms between callbacks): the publish thread gets the
            // context in between (std::mutex is not fair; back-to-back updates would starve it)
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
        done = true;
    });
    std::thread publish([&] {
        bool last = false;
        while (!last) {
            last = done.load();
            if (be.refresh(0)) {
                std::lock_guard<std::mutex> lk(be.mirrorMutex());
                const auto &L = be.level(0);
                seen.emplace_back(L.update_index,
                                  fnv(L.update.data(), 4 * cells, fnv(L.logodds.data(), 4 * cells)));
            }
        }
    });
    spin.join();
    publish.join();

    for (int k = 0; k < 3 * K; ++k)
        if (memcmp(&gpose[k], &opose[k], 4) != 0) {
            fprintf(stderr, "pose mismatch at scan %d: %.9g vs %.9g\n", k / 3, gpose[k], opose[k]);
            ++errors;
            break;
        }
    int prev = -3, distinct = 0;
    for (const auto &s : seen) {
        if (s.first < prev) {
            fprintf(stderr, "update index went back: %d after %d\n", s.first, prev);
            ++errors;
        }
        if (s.first != prev) ++distinct;
        prev = s.first;
        auto it = want.find(s.first);
        if (it == want.end() || it->second != s.second) {
            fprintf(stderr, "snapshot with update index %d differs from the oracle's map\n", s.first);
            ++errors;
        }
    }
    if (seen.empty() || seen.back().first != K - 1) {
        fprintf(stderr, "final snapshot index %d, expected %d\n", seen.empty() ? -9 : seen.back().first, K - 1);
        ++errors;
    }
    if (distinct < 3) {
        fprintf(stderr, "the publish thread saw only %d distinct maps\n", distinct);
        ++errors;
    }
    printf("scans %d snapshots %zu distinct update indices %d errors %d\n", K, seen.size(), distinct, errors);
    return errors ? 1 : 0;
}
