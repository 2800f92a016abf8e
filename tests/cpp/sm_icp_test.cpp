// tests/cpp/sm_icp_test.cpp -- TEST INFRASTRUCTURE.  The lesson3 drop-in `slam2d_sm_icp(&input_, &output_)`
// (include/slam2d/sm_icp_hip.h) driven exactly as plicp_odometry.cc drives CSM's sm_icp:
//   * LaserScanToLDP (plicp_odometry.cc:285-322): valid / readings by range_min < r < range_max (else -1),
//     theta[i] = scan.angle_min + i * scan.angle_increment evaluated in FLOAT (LaserScan's float32
//     fields), min_theta / max_theta = theta[0] / theta[n-1];
//   * the node's parameter values (:74-186) written into sm_params fields, first_guess per pair;
// checked against the C restatement oracle/plicp_oracle.c (plo_icp_theta, the kernel's reduction
// order): valid, iterations, nvalid and every bit of x and error.
//
// CSM itself is absent: the structs below carry the field names CSM's algos.h / laser_data.h document,
// which is all sm_icp_hip.h reads (it is a template over the node's own struct types).
//
// usage: sm_icp_test <pairs.bin>
//   pairs.bin: int32 K, int32 n, float32 angle_min, float32 angle_increment, float32 range_min,
//              float32 range_max, float32 ranges[K + 1][n], float64 guess[K][3]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

struct laser_data {
    int nrays;
    double min_theta, max_theta;
    double *theta;
    int *valid;
    double *readings;
};
typedef laser_data *LDP;
struct sm_params {
    LDP laser_ref, laser_sens;
    double first_guess[3];
    double max_angular_correction_deg, max_linear_correction;
    int max_iterations;
    double epsilon_xy, epsilon_theta, max_correspondence_dist, sigma;
    int use_corr_tricks, restart;
    double restart_threshold_mean_error, restart_dt, restart_dtheta, clustering_threshold;
    int orientation_neighbourhood, use_point_to_line_distance, do_alpha_test;
    double do_alpha_test_thresholdDeg, outliers_maxPerc, outliers_adaptive_order, outliers_adaptive_mult;
    int do_visibility_test, outliers_remove_doubles, do_compute_covariance, debug_verify_tricks, use_ml_weights,
        use_sigma_weights;
};
struct sm_result {
    int valid;
    double x[3];
    int iterations, nvalid;
    double error;
};

#include <slam2d/sm_icp_hip.h>

extern "C" {  // oracle/plicp_oracle.c
typedef struct {
    double max_angular_correction_deg, max_linear_correction, epsilon_xy, epsilon_theta, max_correspondence_dist,
        outliers_maxPerc, outliers_adaptive_order, outliers_adaptive_mult;
    int max_iterations, use_point_to_line_distance, outliers_remove_doubles, pad_;
} plo_params;
int plo_icp_theta(const plo_params *p, int n, double angle_min, double angle_inc, const double *theta,
                  const double *ref_r, const double *sens_r, const double *first_guess, int reduce_threads,
                  double *x_out, int *iterations_out, int *nvalid_out, double *error_out, int *trace_hashes);
}

static void to_ldp(const float *ranges, int n, float amin, float ainc, float rmin, float rmax, laser_data &l,
                   std::vector<double> &th, std::vector<int> &val, std::vector<double> &rd)
{
    th.resize(n);
    val.resize(n);
    rd.resize(n);
    for (unsigned int i = 0; i < (unsigned)n; i++) {
        const double r = ranges[i];
        if (r > rmin && r < rmax) {
            val[i] = 1;
            rd[i] = r;
        } else {
            val[i] = 0;
            rd[i] = -1;
        }
        th[i] = amin + i * ainc;  // float arithmetic, as plicp_odometry.cc:306 on LaserScan's float32 fields
    }
    l.nrays = n;
    l.theta = th.data();
    l.valid = val.data();
    l.readings = rd.data();
    l.min_theta = th[0];
    l.max_theta = th[n - 1];
}

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t K = 0, n = 0;
    float amin, ainc, rmin, rmax;
    if (fread(&K, 4, 1, f) != 1 || fread(&n, 4, 1, f) != 1 || fread(&amin, 4, 1, f) != 1 ||
        fread(&ainc, 4, 1, f) != 1 || fread(&rmin, 4, 1, f) != 1 || fread(&rmax, 4, 1, f) != 1)
        return 2;
    std::vector<float> ranges((size_t)(K + 1) * n);
    std::vector<double> guess((size_t)K * 3);
    if (fread(ranges.data(), 4, ranges.size(), f) != ranges.size() || fread(guess.data(), 8, guess.size(), f) != guess.size())
        return 2;
    fclose(f);

    sm_params in;
    memset(&in, 0, sizeof(in));
    in.max_angular_correction_deg = 45.0;  // ScanMatchPLICP::InitParams defaults (plicp_odometry.cc:74-186)
    in.max_linear_correction = 1.0;
    in.max_iterations = 10;
    in.epsilon_xy = 0.000001;
    in.epsilon_theta = 0.000001;
    in.max_correspondence_dist = 1.0;
    in.sigma = 0.010;
    in.use_corr_tricks = 1;
    in.clustering_threshold = 0.25;
    in.orientation_neighbourhood = 20;
    in.use_point_to_line_distance = 1;
    in.outliers_maxPerc = 0.90;
    in.outliers_adaptive_order = 0.7;
    in.outliers_adaptive_mult = 2.0;
    in.outliers_remove_doubles = 1;
    plo_params op = {45.0, 1.0, 0.000001, 0.000001, 1.0, 0.90, 0.7, 2.0, 10, 1, 1, 0};

    int errors = 0, valid = 0;
    laser_data lref, lsens;
    std::vector<double> th0, th1, rd0, rd1;
    std::vector<int> v0, v1;
    for (int k = 0; k < K; ++k) {
        to_ldp(&ranges[(size_t)k * n], n, amin, ainc, rmin, rmax, lref, th0, v0, rd0);
        to_ldp(&ranges[(size_t)(k + 1) * n], n, amin, ainc, rmin, rmax, lsens, th1, v1, rd1);
        in.laser_ref = &lref;
        in.laser_sens = &lsens;
        for (int c = 0; c < 3; ++c) in.first_guess[c] = guess[3 * k + c];
        sm_result out;
        memset(&out, 0, sizeof(out));
        slam2d_sm_icp(&in, &out);  // the one-call drop-in of sm_icp(&input_, &output_) (:391)

        double x[3], err = 0.0;
        int it = 0, nv = 0, hashes[64];
        const int ok = plo_icp_theta(&op, n, th0[0], 0.0, th0.data(), rd0.data(), rd1.data(), in.first_guess, 256, x,
                                     &it, &nv, &err, hashes);
        valid += out.valid;
        if (out.valid != ok || out.iterations != it || out.nvalid != nv || memcmp(out.x, x, sizeof x) != 0 ||
            memcmp(&out.error, &err, sizeof err) != 0) {
            fprintf(stderr, "pair %d: device (%d, %d it, %d nvalid, %.17g %.17g %.17g) vs oracle (%d, %d, %d, %.17g %.17g %.17g)\n",
                    k, out.valid, out.iterations, out.nvalid, out.x[0], out.x[1], out.x[2], ok, it, nv, x[0], x[1], x[2]);
            ++errors;
        }
    }
    // an unsupported switch must not silently run: output->valid = 0
    in.do_compute_covariance = 1;
    sm_result bad;
    bad.valid = 7;
    slam2d_sm_icp(&in, &bad);
    if (bad.valid != 0) {
        fprintf(stderr, "do_compute_covariance accepted\n");
        ++errors;
    }
    printf("pairs %d valid %d errors %d\n", K, valid, errors);
    return errors || valid == 0 ? 1 : 0;
}
