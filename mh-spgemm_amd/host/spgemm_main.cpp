// spgemm_main.cpp -- the `spgemm <file.mtx>` driver (reference src/main.cu:74-217)
// on top of the C-ABI, printing the reference's stdout lines.
//
//   spgemm [--iters K] [--warmup W] <file.mtx>
//
// Flow as in the reference: read (mmio semantics), reject non-square A (exit 0,
// main.cu:92-96), B = A, count intermediate products on the host (:102-107),
// H2D, run MH_spgemm, print per-phase times and GFLOPS = 2*flop/getTotal().
// Differences: W untimed warm-up calls (the reference warms the GPU with an
// empty kernel, MH_spgemm.cuh:10-25), K timed calls averaged (reference iter=1),
// and an extra e2e line that includes Form_mask_matrix_B.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "mh_spgemm.hpp"

static std::string extract_matrix_name(const std::string& path) {
    const size_t s = path.find_last_of("/\\");
    std::string f = s == std::string::npos ? path : path.substr(s + 1);
    const size_t d = f.find_last_of('.');
    return d == std::string::npos ? f : f.substr(0, d);
}

int main(int argc, char** argv) {
    int iters = 1, warmup = 1;
    const char* filename = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) iters = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--warmup") && i + 1 < argc) warmup = std::atoi(argv[++i]);
        else if (!filename) filename = argv[i];
        else filename = nullptr, i = argc;
    }
    if (!filename || iters < 1 || warmup < 0) {
        std::puts("Invalid Arguments.");
        std::puts("Usage:\t ./spgemm [--iters K] [--warmup W] <Input File>");
        return -1;
    }
    const std::string matrix_name = extract_matrix_name(filename);
    CSR A, B, C;
    if (readMtxFile(A, filename) != 0) return -1;
    if (A.M != A.N) {
        std::puts("C=AA must have rowA = colA. Exit.");
        return 0;
    }
    std::printf("--------------------------SpGEMM Start!!!--------------------------\n");
    B = A;
    const unsigned long long int_result = mhs_flop_count(A.nnz, A.col, B.ptr);
    double Gflops = 0;
    try {
        A.H2D();
        // B = A: share A's device arrays (C = A*A), no second copy.
        B.d_ptr = A.d_ptr;
        B.d_col = A.d_col;
        B.d_val = A.d_val;
        std::printf("Matrix %s (%d , %d) nnz:%d\n", matrix_name.c_str(), A.M, B.N, A.nnz);
        std::printf("SpGEMM intermediate result = %lld\n", (long long)int_result);
        Tool tools;
        Timing timing, bench;
        for (int i = 0; i < warmup; ++i) {
            MH_spgemm(A, B, C, timing, tools);
            mhs_csr c{C.M, C.N, C.nnz, C.d_ptr, C.d_col, C.d_val};
            mhs_ctx_recycle(tools.ctx, &c);
            C.d_ptr = C.d_col = nullptr;
            C.d_val = nullptr;
        }
        for (int i = 0; i < iters; ++i) {
            MH_spgemm(A, B, C, timing, tools);
            bench += timing;
            if (i < iters - 1) {
                mhs_csr c{C.M, C.N, C.nnz, C.d_ptr, C.d_col, C.d_val};
                mhs_ctx_recycle(tools.ctx, &c);
                C.d_ptr = C.d_col = nullptr;
                C.d_val = nullptr;
            }
        }
        bench /= iters;
        bench.print_step_time();
        Gflops = 2.0 * (double)int_result / (bench.getTotal() * 1e6);
        std::printf("MH-SpGEMM runtime is %.3lfms, Gflops is %.2lf\n", bench.getTotal(), Gflops);
        std::printf("MH-SpGEMM e2e (incl. form_mask_matrix_B) is %.3lfms, Gflops is %.2lf\n", bench.total_e2e,
                    2.0 * (double)int_result / (bench.total_e2e * 1e6));
        C.d_release_csr();
        B.d_ptr = B.d_col = nullptr;
        B.d_val = nullptr;
    } catch (const std::exception&) {
        std::printf("MH-SpGEMM failed!!!\n");
        B.d_ptr = B.d_col = nullptr;
        B.d_val = nullptr;
    }
    std::printf("--------------------------SpGEMM   End!!!--------------------------\n");
    return 0;
}
