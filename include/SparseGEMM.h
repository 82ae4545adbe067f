/*
 * SparseGEMM.h -- drop-in for the reference's header-only template API
 * (/root/reference/SparseGEMM.h, used by SparseGEMM.cpp), SURVEY.md §8a rows a8/a9.
 *
 * Same names, template parameters and parameter types, so SparseGEMM.cpp
 * compiles against this header unchanged (oracle/Makefile target
 * `sparsegemm`) and deduces the same function-pointer types in its
 * measure_cycles(sparseGEMM, ...) calls (SparseGEMM.cpp:149-156):
 *
 *   SparseFormat                   SparseGEMM.h:13-40   -> tcsc_sparse_format (host, row-major walk)
 *   initX<T>                       SparseGEMM.h:42-51   data generation, host
 *   generateSparseMatrix<T>        SparseGEMM.h:53-102  data generation, host
 *   sparseGEMM<T>                  SparseGEMM.h:104-119 -> tcsc_sparse_gemm       (gfx950 gather)
 *   GEMM<T>                        SparseGEMM.h:121-133 -> tcsc_dense_gemm        (rocBLAS fp32)
 *   GEMM_PReLU<T>                  SparseGEMM.h:135-149 -> tcsc_dense_gemm_prelu  (rocBLAS fp32)
 *   sparseGEMM_PReLU<T>            SparseGEMM.h:151-168 -> tcsc_sparse_gemm_prelu (gfx950 gather)
 *   compare_results<T>             SparseGEMM.h:171-184 host check, same 10e-6 tolerance and message
 *
 * The compute templates run on the GPU in fp32, so they exist for T = float
 * only: any other T fails to compile (static_assert) rather than silently
 * running a CPU loop.  The reference puts `using namespace std;` in its
 * header and SparseGEMM.cpp relies on it (vector, cout, fill); so does this one.
 * Link with -ltcsc_amd.  See include/sparse_gemm.h for the runtime contract.
 */
#pragma once

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <ctime>
#include <iostream>
#include <random>
#include <type_traits>
#include <vector>

#include "sparse_gemm.h"

using namespace std;

/* Ternary int matrix (K x N, row-major) in TCSC form: >= 1 -> +1 rows,
 * <= -1 -> -1 rows, ascending per column; col_start_* hold N+1 offsets. */
class SparseFormat {
public:
    vector<int> col_start_pos;
    vector<int> col_start_neg;
    vector<int> row_index_pos;
    vector<int> row_index_neg;

    SparseFormat(int* matrix, int K, int N) : col_start_pos(N + 1), col_start_neg(N + 1) {
        int n_pos = 0, n_neg = 0;
        if (tcsc_sparse_format(matrix, K, N, col_start_pos.data(), col_start_neg.data(), nullptr, nullptr, &n_pos,
                               &n_neg) != 0) {
            cerr << "SparseFormat: bad matrix (K=" << K << ", N=" << N << ")" << endl;
            abort();
        }
        row_index_pos.resize(n_pos);
        row_index_neg.resize(n_neg);
        // data() of an empty vector may be NULL; the builder wants both arrays
        int dummy[2];
        tcsc_sparse_format(matrix, K, N, col_start_pos.data(), col_start_neg.data(),
                           n_pos ? row_index_pos.data() : dummy, n_neg ? row_index_neg.data() : dummy + 1, &n_pos,
                           &n_neg);
    }
};

/* LEN values drawn uniformly from the integers in [-Range, Range], from a
 * generator seeded with the wall clock (as the reference does). */
template <typename T>
vector<T> initX(int LEN, int Range) {
    mt19937 gen(static_cast<unsigned int>(time(0)));
    uniform_int_distribution<int> pick(-Range, Range);
    vector<T> X(LEN);
    for (auto& x : X) x = pick(gen);
    return X;
}

/* H x W ternary matrix with about W / nonZero nonzeros per row.
 * uniformDistribution: per 2*nonZero-wide window of a row, one +1 and one -1
 * at distinct even offsets (rand() % nonZero * 2, as written in the reference).
 * Otherwise: per row, W/nonZero/2 + v entries of +1 and W/nonZero/2 - v of
 * -1 at distinct random positions, v ~ U{0 .. W/nonZero/20 + 1}. */
template <typename T>
vector<T> generateSparseMatrix(int H, int W, int nonZero, bool uniformDistribution) {
    vector<T> out((size_t)H * W, 0);
    if (uniformDistribution) {
        const int span = nonZero * 2;
        for (int h = 0; h < H; h++) {
            T* row = out.data() + (size_t)h * W;
            for (int w = 0; w < W; w += span) {
                const int up = rand() % nonZero * 2;
                int down = rand() % nonZero * 2;
                while (down == up) down = rand() % nonZero * 2;
                // the reference writes past the row (and, on the last row,
                // past the matrix) when W is not a multiple of 2*nonZero
                if (w + up < W) row[w + up] = 1;
                if (w + down < W) row[w + down] = -1;
            }
        }
        return out;
    }
    mt19937 gen(static_cast<unsigned int>(time(0)));
    uniform_int_distribution<int> col(0, W - 1);
    uniform_int_distribution<int> skew(0, int(W / nonZero / 20 + 1));
    auto scatter = [&](T* row, int count, T value) {  // `count` distinct empty slots
        for (int placed = 0; placed < count;) {
            const int c = col(gen);
            if (row[c] == 0) {
                row[c] = value;
                ++placed;
            }
        }
    };
    for (int h = 0; h < H; h++) {
        T* row = out.data() + (size_t)h * W;
        const int v = skew(gen), half = (W / nonZero) / 2;
        scatter(row, half + v, 1);
        scatter(row, half - v, -1);
    }
    return out;
}

template <typename T>
void sparseGEMM(T* X, int* col_start_pos, int* col_start_neg, int* row_index_pos, int* row_index_neg, T* b, T* Y,
                int M, int N, int K) {
    static_assert(std::is_same<T, float>::value, "sparseGEMM: the gfx950 path computes in fp32 (T = float)");
    tcsc_sparse_gemm(X, col_start_pos, col_start_neg, row_index_pos, row_index_neg, b, Y, M, N, K);
}

template <typename T>
void GEMM(T* X, T* W, T* b, T* Y, int M, int N, int K) {
    static_assert(std::is_same<T, float>::value, "GEMM: the GPU dense baseline is fp32 (T = float)");
    tcsc_dense_gemm(X, W, b, Y, M, N, K);
}

template <typename T>
void GEMM_PReLU(T* X, T* W, T* b, T* Y, int M, int N, int K, T a) {
    static_assert(std::is_same<T, float>::value, "GEMM_PReLU: the GPU dense baseline is fp32 (T = float)");
    tcsc_dense_gemm_prelu(X, W, b, Y, M, N, K, a);
}

template <typename T>
void sparseGEMM_PReLU(T* X, int* col_start_pos, int* col_start_neg, int* row_index_pos, int* row_index_neg, T* b,
                      T* Y, int M, int N, int K, T a) {
    static_assert(std::is_same<T, float>::value, "sparseGEMM_PReLU: the gfx950 path computes in fp32 (T = float)");
    tcsc_sparse_gemm_prelu(X, col_start_pos, col_start_neg, row_index_pos, row_index_neg, b, Y, M, N, K, a);
}

/* First element with |result - groundTruth| > 10e-6 is printed and fails the
 * check (SparseGEMM.h:176: the literal is 1e-5). */
template <typename T>
bool compare_results(T* result, T* groundTruth, int H, int W) {
    const size_t n = (size_t)H * W;
    for (size_t i = 0; i < n; ++i) {
        if (abs(result[i] - groundTruth[i]) > 10e-6) {
            cout << "Error at: H=" << i / W << ", W=" << i % W << ", result=" << result[i]
                 << ", groundTruth=" << groundTruth[i] << endl;
            return false;
        }
    }
    return true;
}
