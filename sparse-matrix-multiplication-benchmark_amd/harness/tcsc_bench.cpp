// tcsc_bench -- native benchmark driver for libtcsc_amd.so.
//
// The counterpart of the reference harness main.cpp (main.cpp:252-456): the
// same cases, the same validate-then-measure sequence, the same result table
// and the same six legacy "NAME cycles=..., flops=..., performance=..." lines
// per case (main.cpp:409-432), so out.txt files written by either program
// parse alike (harness/out2csv.py).  It adds what a GPU run needs:
//
//   --api device  (default) inputs resident in HBM, one plan per case, every
//                 launch bracketed by hipEvents on its stream; reports kernel
//                 time, G-add-ops/s and the HBM roofline fraction.
//   --api host    the drop-in host-pointer entry points (sparse/tcsc.h), i.e.
//                 what the reference's main.cpp measures when it is linked
//                 against this library: PCIe transfers included, timed with
//                 the reference's own protocol (measure.h:13-76: NUM_RUNS
//                 scaled until a pass covers CYCLES_REQUIRED TSC cycles, then
//                 the mean over REP passes).
//   --json FILE / --csv FILE   one record per (case, algorithm).
//
// Cases: --cases reference (main.cpp:258-264, 50 % sparsity via
// init_rand_sparse(K, N, 2), main.cpp:278), --config 1..5 (BASELINE.json,
// SURVEY.md §8d) or --shape M,K,N,NZ (NZ as init_rand_sparse's non_zero:
// density 1/NZ).  Inputs come from the library's seeded generators
// (dense/dense.h), seed 0x7C5C0000 + case index unless --seed is given.
//
// Validation (as main.cpp:317-366, exit(1) on a mismatch): every TCSC
// variant against the dense baseline of the same variant
// (tcsc_gpu_dense_sgemm, fp32 rocBLAS SGEMM).  The reference's 1e-4 absolute
// tolerance (dense.c:43) is too tight at the large configs,
// so the bound is per element: |y - y_dense| <= max(1, a) * 2^-19 * S, with
// S = |B| + |X| . |W| (the sum of the magnitudes of the terms), itself
// computed by the dense path.  Both results carry rounding error, hence 2^-19
// (two budgets of the 2^-20 oracle bound).
//
// Cycles in the legacy lines are host TSC cycles (calibrated against
// CLOCK_MONOTONIC), so "performance" keeps the reference's flops-per-cycle
// meaning; flops are the reference's count, 2*M*nnz + M*N
// (main.cpp:47-51) and 2*M*N*K + M*N for the dense GEMM (main.cpp:293).
#include <hip/hip_runtime.h>
#include <x86intrin.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "dense/dense.h"
#include "sparse/tcsc.h"
#include "tcsc_gpu.h"

namespace {

constexpr unsigned long long kSeed0 = 0x7C5C0000ull;
constexpr double kHbmPeak = 8.0e12;  // MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
constexpr float kAlpha = 0.2f;       // main.cpp:268

struct Case {
    std::string name;
    int M, K, N, nz;
    unsigned long long seed;
};

struct Options {
    std::vector<Case> cases;
    std::string api = "device";
    std::string json, csv;
    int warmup = 5, reps = 50, device = 0;
    bool have_seed = false, dense = true, validate = true, quiet = false, reference_order = false;
    unsigned long long seed = 0;
    // host protocol (measure.h): NUM_RUNS, CYCLES_REQUIRED, REP (main.cpp:9-15)
    int num_runs = 20, rep = 50;
    double cycles_required = 1e8;
};

// algorithms in the order of the legacy lines (main.cpp:409-432)
struct Algo {
    const char* legacy;  // legacy line name, padded as main.cpp prints it
    const char* key;     // record name
    int variant;         // enum tcsc_variant, -1 = dense GEMM
};
const Algo kAlgos[] = {
    {"GEMM        ", "dense_gemm", -1},
    {"TCSC_basic  ", "basic", TCSC_VARIANT_BASIC},
    {"TCSC_opt    ", "optimized", TCSC_VARIANT_OPTIMIZED},
    {"TCSC_PReLU_basic", "prelu_basic", TCSC_VARIANT_PRELU_BASIC},
    {"TCSC_PReLU_sep  ", "prelu_separate", TCSC_VARIANT_PRELU_SEPARATE},
    {"TCSC_PReLU_otg  ", "prelu_onthego", TCSC_VARIANT_PRELU_ONTHEGO},
};
constexpr int kNumAlgos = sizeof(kAlgos) / sizeof(kAlgos[0]);

struct Result {
    double ms_median = 0, ms_mean = 0, ms_min = 0;  // per call
    double cycles = 0;                              // TSC cycles per call
    long long flops = 0;
    double add_ops = 0, bytes = 0;
    double worst_err_over_bound = 0;
    bool measured = false;
};

[[noreturn]] void die(const char* what) {
    std::fprintf(stderr, "tcsc_bench: %s\n", what);
    std::exit(2);
}

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "tcsc_bench: %s: %s\n", what, hipGetErrorString(e));
        std::exit(2);
    }
}

void lib_ok(int status, const char* what) {
    if (status != TCSC_OK) {
        std::fprintf(stderr, "tcsc_bench: %s failed (%d): %s\n", what, status, tcsc_gpu_last_error());
        std::exit(2);
    }
}

double monotonic_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

// TSC ticks per second, measured over ~100 ms
double tsc_hz() {
    const double t0 = monotonic_s();
    const unsigned long long c0 = __rdtsc();
    while (monotonic_s() - t0 < 0.1) {
    }
    const unsigned long long c1 = __rdtsc();
    return (double)(c1 - c0) / (monotonic_s() - t0);
}

void usage() {
    std::printf(
        "usage: tcsc_bench [--cases reference] [--config 1..5]... [--shape M,K,N,NZ]...\n"
        "                  [--api device|host] [--warmup W] [--reps R] [--device D] [--seed S]\n"
        "                  [--order fast|reference] [--no-dense] [--no-validate]\n"
        "                  [--num-runs N] [--rep R] [--cycles-required C] [--json FILE] [--csv FILE] [--quiet]\n"
        "defaults: --cases reference --api device (main.cpp's five cases)\n");
}

Case baseline_config(int idx) {
    // BASELINE.json configs; NZ = 1/density (utils.h:36-43)
    switch (idx) {
        case 1: return {"cfg1", 128, 256, 256, 10, kSeed0 + 1};
        case 2: return {"cfg2", 1024, 4096, 4096, 20, kSeed0 + 2};
        case 3: return {"cfg3", 1024, 4096, 4096, 20, kSeed0 + 3};
        case 4: return {"cfg4", 4096, 16384, 16384, 50, kSeed0 + 4};
        case 5: return {"cfg5", 2048, 8192, 8192, 2, kSeed0 + 5};
    }
    die("--config takes 1..5");
}

Options parse(int argc, char** argv) {
    Options o;
    auto need = [&](int& i) -> const char* {
        if (i + 1 >= argc) {
            usage();
            die("missing value");
        }
        return argv[++i];
    };
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--cases") {
            const std::string v = need(i);
            if (v != "reference") die("--cases takes 'reference'");
            // main.cpp:258-264, (M, K, N), init_rand_sparse(K, N, 2)
            const int shapes[5][3] = {{1, 512, 2048}, {1, 1024, 4096}, {1, 2048, 8192}, {256, 512, 2048}, {256, 1024, 4096}};
            for (int c = 0; c < 5; ++c)
                o.cases.push_back({"ref" + std::to_string(c + 1), shapes[c][0], shapes[c][1], shapes[c][2], 2,
                                   kSeed0 + 100 + (unsigned long long)c});
        } else if (a == "--config") {
            o.cases.push_back(baseline_config(std::atoi(need(i))));
        } else if (a == "--shape") {
            Case c{};
            if (std::sscanf(need(i), "%d,%d,%d,%d", &c.M, &c.K, &c.N, &c.nz) != 4 || c.M < 1 || c.K < 1 || c.N < 1 ||
                c.nz < 1)
                die("--shape takes M,K,N,NZ (all >= 1)");
            c.name = "shape" + std::to_string(o.cases.size() + 1);
            c.seed = kSeed0 + 200 + o.cases.size();
            o.cases.push_back(c);
        } else if (a == "--api") {
            o.api = need(i);
            if (o.api != "device" && o.api != "host") die("--api takes device or host");
        } else if (a == "--warmup") {
            o.warmup = std::max(0, std::atoi(need(i)));
        } else if (a == "--reps") {
            o.reps = std::max(1, std::atoi(need(i)));
        } else if (a == "--device") {
            o.device = std::atoi(need(i));
        } else if (a == "--seed") {
            o.have_seed = true;
            o.seed = std::strtoull(need(i), nullptr, 0);
        } else if (a == "--order") {
            const std::string v = need(i);
            if (v != "fast" && v != "reference") die("--order takes fast or reference");
            o.reference_order = v == "reference";
        } else if (a == "--no-dense") {
            o.dense = false;
        } else if (a == "--no-validate") {
            o.validate = false;
        } else if (a == "--num-runs") {
            o.num_runs = std::max(1, std::atoi(need(i)));
        } else if (a == "--rep") {
            o.rep = std::max(1, std::atoi(need(i)));
        } else if (a == "--cycles-required") {
            o.cycles_required = std::atof(need(i));
        } else if (a == "--json") {
            o.json = need(i);
        } else if (a == "--csv") {
            o.csv = need(i);
        } else if (a == "--quiet") {
            o.quiet = true;
        } else if (a == "-h" || a == "--help") {
            usage();
            std::exit(0);
        } else {
            usage();
            die(("unknown option " + a).c_str());
        }
    }
    if (o.cases.empty()) {
        const char* one[] = {"tcsc_bench", "--cases", "reference"};
        o.cases = parse(3, const_cast<char**>(one)).cases;
    }
    if (o.have_seed)
        for (size_t c = 0; c < o.cases.size(); ++c) o.cases[c].seed = o.seed + c;
    if (o.validate && !o.dense) die("validation needs the dense baseline (drop --no-dense or add --no-validate)");
    return o;
}

struct DevBuf {
    void* p = nullptr;
    explicit DevBuf(size_t bytes) { hip_ok(hipMalloc(&p, bytes ? bytes : 4), "hipMalloc"); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    float* f() const { return static_cast<float*>(p); }
    int* i() const { return static_cast<int*>(p); }
};

// Times `launch` (enqueues one call on `s`) with hipEvents around each call.
template <class F>
Result time_device(F launch, hipStream_t s, int warmup, int reps, double hz) {
    for (int w = 0; w < warmup; ++w) launch();
    hip_ok(hipStreamSynchronize(s), "warmup");
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto& e : ev) hip_ok(hipEventCreate(&e), "hipEventCreate");
    hip_ok(hipEventRecord(ev[0], s), "hipEventRecord");
    for (int r = 0; r < reps; ++r) {
        launch();
        hip_ok(hipEventRecord(ev[r + 1], s), "hipEventRecord");
    }
    hip_ok(hipEventSynchronize(ev[reps]), "hipEventSynchronize");
    std::vector<double> ms(reps);
    for (int r = 0; r < reps; ++r) {
        float t = 0;
        hip_ok(hipEventElapsedTime(&t, ev[r], ev[r + 1]), "hipEventElapsedTime");
        ms[r] = t;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    Result res;
    std::vector<double> sorted = ms;
    std::sort(sorted.begin(), sorted.end());
    res.ms_median = reps % 2 ? sorted[reps / 2] : 0.5 * (sorted[reps / 2 - 1] + sorted[reps / 2]);
    res.ms_min = sorted[0];
    double sum = 0;
    for (double v : ms) sum += v;
    res.ms_mean = sum / reps;
    res.cycles = res.ms_median * 1e-3 * hz;
    res.measured = true;
    return res;
}

// measure.h:13-76 / main.cpp:54-113 with TSC cycles (x86 path)
template <class F>
Result time_host(F call, const Options& o, double hz) {
    int num_runs = o.num_runs;
    double multiplier = 1.0;
    do {
        num_runs = std::max(1, (int)(num_runs * multiplier));
        const unsigned long long t0 = __rdtsc();
        for (int i = 0; i < num_runs; ++i) call();
        const double cycles = (double)(__rdtsc() - t0);
        multiplier = o.cycles_required / cycles;
    } while (multiplier > 2);
    double total = 0, best = 1e300;
    for (int j = 0; j < o.rep; ++j) {
        const unsigned long long t0 = __rdtsc();
        for (int i = 0; i < num_runs; ++i) call();
        const double c = (double)(__rdtsc() - t0) / num_runs;
        total += c;
        best = std::min(best, c);
    }
    Result res;
    res.cycles = total / o.rep;
    res.ms_mean = res.ms_median = res.cycles / hz * 1e3;  // the protocol keeps only the mean
    res.ms_min = best / hz * 1e3;
    res.measured = true;
    return res;
}

// worst |y - ref| / (max(1,a) * 2^-19 * S) over the M x N outputs
double worst_ratio(const std::vector<float>& y, const std::vector<float>& ref, const std::vector<float>& s, bool prelu) {
    const double scale = (prelu ? std::max(1.0, (double)kAlpha) : 1.0) * std::ldexp(1.0, -19);
    double worst = 0;
    for (size_t i = 0; i < y.size(); ++i) {
        const double bound = scale * (double)s[i];
        const double err = std::fabs((double)y[i] - (double)ref[i]);
        if (std::isnan(y[i]) || std::isnan(ref[i])) {
            if (std::isnan(y[i]) != std::isnan(ref[i])) return INFINITY;
            continue;
        }
        const double r = err == 0 ? 0 : (bound > 0 ? err / bound : INFINITY);
        worst = std::max(worst, r);
    }
    return worst;
}

std::string json_escape(const std::string& s) {
    std::string r;
    for (char c : s) {
        if (c == '"' || c == '\\') r += '\\';
        r += c;
    }
    return r;
}

}  // namespace

int main(int argc, char** argv) {
    Options o = parse(argc, argv);
    setvbuf(stdout, nullptr, _IOLBF, 0);
    if (tcsc_gpu_device_count() < 1) die("no gfx950 device visible (this driver runs the GPU library)");
    hip_ok(hipSetDevice(o.device), "hipSetDevice");
    tcsc_gpu_set_order(o.reference_order ? TCSC_ORDER_REFERENCE : TCSC_ORDER_FAST);
    hipStream_t stream;
    hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    const double hz = tsc_hz();
    hipDeviceProp_t prop;
    hip_ok(hipGetDeviceProperties(&prop, o.device), "hipGetDeviceProperties");

    FILE* jf = o.json.empty() ? nullptr : (o.json == "-" ? stdout : std::fopen(o.json.c_str(), "w"));
    FILE* cf = o.csv.empty() ? nullptr : (o.csv == "-" ? stdout : std::fopen(o.csv.c_str(), "w"));
    if ((!o.json.empty() && !jf) || (!o.csv.empty() && !cf)) die("cannot open the --json/--csv output");
    if (cf)
        std::fprintf(cf,
                     "case,M,K,N,nnz,api,order,algorithm,ms_median,ms_mean,ms_min,cycles,flops,performance,"
                     "g_add_ops_per_s,gb_per_s,hbm_frac,worst_err_over_bound\n");

    std::printf("tcsc_bench: %s (%s, %d CUs), api=%s, order=%s, TSC %.3f GHz, %zu case(s)\n", prop.name,
                prop.gcnArchName, prop.multiProcessorCount, o.api.c_str(), o.reference_order ? "reference" : "fast",
                hz * 1e-9, o.cases.size());

    for (size_t ci = 0; ci < o.cases.size(); ++ci) {
        const Case& c = o.cases[ci];
        const int M = c.M, K = c.K, N = c.N;
        std::printf("\n+----------------------------------------------------------------------+\n");
        std::printf("|  [TEST %zu/%zu] Matrix Size: %dx%dx%d (Sparsity: %.0f%%)\n", ci + 1, o.cases.size(), M, K, N,
                    100.0 * (1.0 - 1.0 / c.nz));
        std::printf("+----------------------------------------------------------------------+\n");

        // inputs from the library's seeded generators (dense/dense.h)
        tcsc_set_seed(c.seed);
        float* X = init_rand_dense(M, K);
        float* B = init_rand_dense(N, 1);
        float* Wd = init_rand_sparse(K, N, c.nz);
        if (!X || !B || !Wd) die("host allocation failed");
        const size_t nX = (size_t)M * K, nW = (size_t)K * N, nY = (size_t)M * N;

        DevBuf dX(nX * 4), dB(N * 4), dY(nY * 4), dYd(nY * 4);
        hip_ok(hipMemcpy(dX.p, X, nX * 4, hipMemcpyHostToDevice), "H2D X");
        hip_ok(hipMemcpy(dB.p, B, (size_t)N * 4, hipMemcpyHostToDevice), "H2D B");

        // W: device build (tcsc_gpu_from_dense, bit-exact with tcsc_from_dense)
        tcsc_gpu_plan* plan = nullptr;
        long long nnz = 0;
        std::vector<float> S;  // |B| + |X|.|W| per output, for the validation bound
        std::vector<float> dense_ref[2];  // dense baseline: [0] identity, [1] PReLU
        Result res[kNumAlgos];
        {
            DevBuf dW(nW * 4), csp((size_t)(N + 1) * 4), csn((size_t)(N + 1) * 4);
            hip_ok(hipMemcpy(dW.p, Wd, nW * 4, hipMemcpyHostToDevice), "H2D W");
            int np = 0, nn = 0;
            lib_ok(tcsc_gpu_from_dense(dW.f(), K, N, csp.i(), csn.i(), nullptr, nullptr, &np, &nn, stream),
                   "tcsc_gpu_from_dense (count)");
            DevBuf rip((size_t)std::max(np, 1) * 4), rin((size_t)std::max(nn, 1) * 4);
            lib_ok(tcsc_gpu_from_dense(dW.f(), K, N, csp.i(), csn.i(), rip.i(), rin.i(), &np, &nn, stream),
                   "tcsc_gpu_from_dense");
            nnz = (long long)np + nn;
            if (o.api == "device") {
                lib_ok(tcsc_gpu_plan_create_device(K, N, csp.i(), csn.i(), rip.i(), rin.i(), 0, N, o.device, stream,
                                                   &plan),
                       "tcsc_gpu_plan_create_device");
                lib_ok(tcsc_gpu_plan_reserve(plan, M), "tcsc_gpu_plan_reserve");
            }
            std::printf("[*] Matrix info: %lld non-zeros out of %lld elements\n", nnz, (long long)K * N);

            if (o.dense) {
                // dense baseline: validation reference and the "Dense GEMM" line
                for (int pr = 0; pr < (o.validate ? 2 : 0); ++pr) {
                    lib_ok(tcsc_gpu_dense_sgemm(dX.f(), dW.f(), dB.f(), dYd.f(), M, N, K, N,
                                                pr ? TCSC_VARIANT_PRELU_BASIC : TCSC_VARIANT_BASIC, kAlpha, stream),
                           "tcsc_gpu_dense_sgemm");
                    dense_ref[pr].resize(nY);
                    hip_ok(hipMemcpyAsync(dense_ref[pr].data(), dYd.p, nY * 4, hipMemcpyDeviceToHost, stream), "D2H");
                    hip_ok(hipStreamSynchronize(stream), "dense");
                }
                res[0] = time_device(
                    [&] {
                        lib_ok(tcsc_gpu_dense_sgemm(dX.f(), dW.f(), dB.f(), dYd.f(), M, N, K, N, TCSC_VARIANT_BASIC,
                                                    kAlpha, stream),
                               "tcsc_gpu_dense_sgemm");
                    },
                    stream, std::min(o.warmup, 3), std::min(o.reps, 10), hz);
                res[0].flops = 2LL * M * N * K + (long long)M * N;  // main.cpp:293
                if (o.validate) {
                    // S = |B| + |X| . |W| via the same dense path on magnitudes
                    std::vector<float> a(std::max(nX, nW));
                    for (size_t i = 0; i < nW; ++i) a[i] = std::fabs(Wd[i]);
                    hip_ok(hipMemcpy(dW.p, a.data(), nW * 4, hipMemcpyHostToDevice), "H2D |W|");
                    for (size_t i = 0; i < nX; ++i) a[i] = std::fabs(X[i]);
                    DevBuf dXa(nX * 4), dBa((size_t)N * 4);
                    hip_ok(hipMemcpy(dXa.p, a.data(), nX * 4, hipMemcpyHostToDevice), "H2D |X|");
                    for (int n = 0; n < N; ++n) a[n] = std::fabs(B[n]);
                    hip_ok(hipMemcpy(dBa.p, a.data(), (size_t)N * 4, hipMemcpyHostToDevice), "H2D |B|");
                    lib_ok(tcsc_gpu_dense_sgemm(dXa.f(), dW.f(), dBa.f(), dYd.f(), M, N, K, N, TCSC_VARIANT_BASIC, 0.f,
                                                stream),
                           "tcsc_gpu_dense_sgemm |.|");
                    S.resize(nY);
                    hip_ok(hipMemcpyAsync(S.data(), dYd.p, nY * 4, hipMemcpyDeviceToHost, stream), "D2H S");
                    hip_ok(hipStreamSynchronize(stream), "abs-sum");
                }
            }
        }

        tcsc_t* W = nullptr;
        if (o.api == "host") {
            W = tcsc_from_dense(Wd, K, N);  // the drop-in builder (tcsc.c:6-66)
            if (!W) die("tcsc_from_dense returned NULL");
        }

        // validation phase (main.cpp:299-368)
        std::vector<float> y(nY);
        const double algo_bytes = 4.0 * ((double)M * K + (double)M * N + (double)nnz + 2.0 * (N + 1) + N);
        for (int ai = 1; ai < kNumAlgos; ++ai) {
            const Algo& al = kAlgos[ai];
            const bool prelu = al.variant >= TCSC_VARIANT_PRELU_BASIC;
            auto host_call = [&](float* Yh) {
                switch (al.variant) {
                    case TCSC_VARIANT_BASIC: tcsc_sgemm_basic(X, W, B, Yh, M, N, K); break;
                    case TCSC_VARIANT_OPTIMIZED: tcsc_sgemm_optimized(X, W, B, Yh, M, N, K); break;
                    case TCSC_VARIANT_PRELU_BASIC: tcsc_sgemm_prelu_basic(X, W, B, kAlpha, Yh, M, N, K); break;
                    case TCSC_VARIANT_PRELU_SEPARATE:
                        tcsc_sgemm_prelu_optimized_separate(X, W, B, kAlpha, Yh, M, N, K);
                        break;
                    default: tcsc_sgemm_prelu_optimized_onthego(X, W, B, kAlpha, Yh, M, N, K); break;
                }
            };
            auto dev_call = [&] {
                lib_ok(tcsc_gpu_sgemm(plan, dX.f(), dB.f(), dY.f(), M, N, al.variant, kAlpha, stream),
                       "tcsc_gpu_sgemm");
            };
            if (o.validate) {
                if (o.api == "host") {
                    host_call(y.data());
                } else {
                    dev_call();
                    hip_ok(hipMemcpyAsync(y.data(), dY.p, nY * 4, hipMemcpyDeviceToHost, stream), "D2H Y");
                    hip_ok(hipStreamSynchronize(stream), "sgemm");
                }
                res[ai].worst_err_over_bound = worst_ratio(y, dense_ref[prelu ? 1 : 0], S, prelu);
                if (!(res[ai].worst_err_over_bound <= 1.0)) {
                    std::printf("[ERROR] %s failed validation!!! (worst error / bound = %g)\n", al.key,
                                res[ai].worst_err_over_bound);
                    std::exit(1);
                }
            }
        }
        if (o.validate) std::printf("[OK] All validation tests passed!\n");

        // performance measurements (main.cpp:370-391)
        std::printf("\n[*] Starting performance measurements...\n");
        for (int ai = 1; ai < kNumAlgos; ++ai) {
            const Algo& al = kAlgos[ai];
            double err = res[ai].worst_err_over_bound;
            if (o.api == "host") {
                res[ai] = time_host(
                    [&] {
                        switch (al.variant) {
                            case TCSC_VARIANT_BASIC: tcsc_sgemm_basic(X, W, B, y.data(), M, N, K); break;
                            case TCSC_VARIANT_OPTIMIZED: tcsc_sgemm_optimized(X, W, B, y.data(), M, N, K); break;
                            case TCSC_VARIANT_PRELU_BASIC:
                                tcsc_sgemm_prelu_basic(X, W, B, kAlpha, y.data(), M, N, K);
                                break;
                            case TCSC_VARIANT_PRELU_SEPARATE:
                                tcsc_sgemm_prelu_optimized_separate(X, W, B, kAlpha, y.data(), M, N, K);
                                break;
                            default: tcsc_sgemm_prelu_optimized_onthego(X, W, B, kAlpha, y.data(), M, N, K); break;
                        }
                    },
                    o, hz);
            } else {
                res[ai] = time_device(
                    [&] {
                        lib_ok(tcsc_gpu_sgemm(plan, dX.f(), dB.f(), dY.f(), M, N, al.variant, kAlpha, stream),
                               "tcsc_gpu_sgemm");
                    },
                    stream, o.warmup, o.reps, hz);
            }
            res[ai].worst_err_over_bound = err;
            res[ai].flops = 2LL * M * nnz + (long long)M * N;  // main.cpp:47-51
            res[ai].add_ops = (double)M * nnz + (double)M * N;
            res[ai].bytes = algo_bytes;
        }

        // result table (main.cpp:198-250)
        if (!o.quiet) {
            std::printf("\n[*] PERFORMANCE RESULTS (%s):\n", o.api == "host" ? "host API, PCIe included" : "device-resident");
            std::printf("+---------------------+-------------+-------------+------------+-------------+---------+\n");
            std::printf("|     Algorithm       |  time (ms)  |    FLOPs    | flops/cyc  | G-add-ops/s | HBM %%   |\n");
            std::printf("+---------------------+-------------+-------------+------------+-------------+---------+\n");
            const char* label[kNumAlgos] = {"Dense GEMM", "TCSC Basic", "TCSC Optimized", "TCSC PReLU Basic",
                                            "TCSC PReLU Separate", "TCSC PReLU OnTheGo"};
            for (int ai = 0; ai < kNumAlgos; ++ai) {
                const Result& r = res[ai];
                if (!r.measured) continue;
                const double s = r.ms_median * 1e-3;
                std::printf("| %-19s | %11.4f | %11lld | %10.4f | %11.1f | %6.2f%% |\n", label[ai], r.ms_median,
                            r.flops, r.flops / r.cycles, ai ? r.add_ops / s * 1e-9 : 0.0,
                            ai ? 100.0 * r.bytes / s / kHbmPeak : 0.0);
            }
            std::printf("+---------------------+-------------+-------------+------------+-------------+---------+\n");
            if (res[0].measured) {
                std::printf("\n[*] SPEEDUP ANALYSIS:\n");
                std::printf("  [1] TCSC Basic vs Dense:         %.2fx faster\n", res[0].cycles / res[1].cycles);
                std::printf("  [2] TCSC Optimized vs Basic:     %.2fx faster\n", res[1].cycles / res[2].cycles);
                std::printf("  [3] Overall Optimization:        %.2fx faster\n", res[0].cycles / res[2].cycles);
                std::printf("  [4] PReLU Separate vs Basic:     %.2fx faster\n", res[3].cycles / res[4].cycles);
                std::printf("  [5] PReLU OnTheGo vs Basic:      %.2fx faster\n", res[3].cycles / res[5].cycles);
            }
        }
        // legacy lines (main.cpp:409-432)
        for (int ai = 0; ai < kNumAlgos; ++ai) {
            const Result& r = res[ai];
            if (!r.measured) continue;
            std::printf("%s cycles=%.0f, flops=%lld, performance=%.4f\n", kAlgos[ai].legacy, r.cycles, r.flops,
                        r.flops / r.cycles);
        }

        for (int ai = 0; ai < kNumAlgos; ++ai) {
            const Result& r = res[ai];
            if (!r.measured) continue;
            const double s = r.ms_median * 1e-3;
            const double gadd = ai ? r.add_ops / s * 1e-9 : 0.0, gbs = ai ? r.bytes / s * 1e-9 : 0.0;
            if (jf)
                std::fprintf(jf,
                             "{\"case\": \"%s\", \"M\": %d, \"K\": %d, \"N\": %d, \"nz\": %d, \"nnz\": %lld, "
                             "\"seed\": %llu, \"api\": \"%s\", \"order\": \"%s\", \"algorithm\": \"%s\", "
                             "\"ms_median\": %.6f, \"ms_mean\": %.6f, \"ms_min\": %.6f, \"cycles\": %.0f, "
                             "\"flops\": %lld, \"performance\": %.4f, \"g_add_ops_per_s\": %.3f, "
                             "\"gb_per_s\": %.3f, \"hbm_frac\": %.5f, \"worst_err_over_bound\": %.4g, "
                             "\"device\": \"%s\"}\n",
                             json_escape(c.name).c_str(), M, K, N, c.nz, nnz, c.seed, o.api.c_str(),
                             o.reference_order ? "reference" : "fast", kAlgos[ai].key, r.ms_median, r.ms_mean,
                             r.ms_min, r.cycles, r.flops, r.flops / r.cycles, gadd, gbs,
                             ai ? gbs * 1e9 / kHbmPeak : 0.0, r.worst_err_over_bound, prop.gcnArchName);
            if (cf)
                std::fprintf(cf, "%s,%d,%d,%d,%lld,%s,%s,%s,%.6f,%.6f,%.6f,%.0f,%lld,%.4f,%.3f,%.3f,%.5f,%.4g\n",
                             c.name.c_str(), M, K, N, nnz, o.api.c_str(), o.reference_order ? "reference" : "fast",
                             kAlgos[ai].key, r.ms_median, r.ms_mean, r.ms_min, r.cycles, r.flops, r.flops / r.cycles,
                             gadd, gbs, ai ? gbs * 1e9 / kHbmPeak : 0.0, r.worst_err_over_bound);
        }

        if (plan) tcsc_gpu_plan_destroy(plan);
        if (W) tcsc_free(W);
        std::free(X);
        std::free(B);
        std::free(Wd);
    }
    if (jf && jf != stdout) std::fclose(jf);
    if (cf && cf != stdout) std::fclose(cf);
    (void)hipStreamDestroy(stream);
    std::printf("\n*** ALL BENCHMARKS COMPLETED! ***\n");
    return 0;
}
