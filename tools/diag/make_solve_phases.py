"""Regenerate tools/diag/solve_phases.patch from the current mvm_lsap_sparse.hip."""
import os, shutil, subprocess
src = open('/root/repo/bpc_baseline_amd/csrc/mvm_lsap_sparse.hip').read()
s = src
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)
rep('''template <typename CT>
__device__ __forceinline__ double sp_block_min(double x, double *s_red, int wave) {''','''__device__ unsigned long long g_sp_phase[4096][10];
#define PH_T() ((long long)__builtin_amdgcn_s_memtime())
#define PH(n) do { tq1 = PH_T(); ph[n] += tq1 - tq0; tq0 = tq1; } while (0)
template <typename CT>
__device__ __forceinline__ double sp_block_min(double x, double *s_red, int wave) {''')
rep('''    int par = 0;
    for (int cur = 0; cur < S; ++cur) {''','''    long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    long long tq0 = PH_T(), tq1;
    int par = 0;
    for (int cur = 0; cur < S; ++cur) {''')
rep('''            if (k > 0) rd = load_row(i, na);''','''            PH(8);
            if (k > 0) rd = load_row(i, na);''')
rep('''            const int lc = rd.lc;
            const CT lv = rd.lv;''','''            const int lc = rd.lc;
            const CT lv = rd.lv;
            if (src.e12) asm volatile("" :: "v"(cv[0]), "v"(lc), "v"(lv));
            PH(0);''')
rep('''            // wave records
            {''','''            asm volatile("" :: "v"(ba), "v"(fr));
            PH(1);
            // wave records
            {''')
rep('''            if (k == 0 && cur + 1 < S) pf = load_row(cur + 1, na);
            __syncthreads();''','''            PH(2);
            if (k == 0 && cur + 1 < S) pf = load_row(cur + 1, na);
            __syncthreads();
            PH(3);''')
rep('''            F = fmin(F, fk);
            lowest = fmin(A, F);''','''            PH(4);
            F = fmin(F, fk);
            lowest = fmin(A, F);''')
rep('''                sink = (int)(fkey & 0xFFFFu);
                sink_ps = 0;''','''                sink = (int)(fkey & 0xFFFFu);
                sink_ps = 0;
                ph[9] += 1;''')
rep('''                sink = (int)(best & 0xFFFF);
                if (t == 0) {''','''                sink = (int)(best & 0xFFFF);
                PH(5);
                if (t == 0) {''')
rep('''        n_steps += k + 1;''','''        PH(6);
        n_steps += k + 1;''')
rep('''    if (t == 0) {
        int32_t *stt = reinterpret_cast<int32_t *>(a.ws + a.ws_offs[p] + y.stats);''','''    PH(7);
    if (t == 0 && p < 4096)
        for (int x = 0; x < 10; ++x) g_sp_phase[p][x] = (unsigned long long)ph[x];
    if (t == 0) {
        int32_t *stt = reinterpret_cast<int32_t *>(a.ws + a.ws_offs[p] + y.stats);''')
rep('''extern "C" {''','''extern "C" {

int mvm_diag_solve_phases(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sp_phase), (size_t)n * 10 * 8) == hipSuccess ? 0 : 1;
}''')
shutil.rmtree('/tmp/dg3', ignore_errors=True)
for d in 'ab':
    os.makedirs(f'/tmp/dg3/{d}/bpc_baseline_amd/csrc')
open('/tmp/dg3/a/bpc_baseline_amd/csrc/mvm_lsap_sparse.hip', 'w').write(src)
open('/tmp/dg3/b/bpc_baseline_amd/csrc/mvm_lsap_sparse.hip', 'w').write(s)
r = subprocess.run(['diff', '-u', 'a/bpc_baseline_amd/csrc/mvm_lsap_sparse.hip', 'b/bpc_baseline_amd/csrc/mvm_lsap_sparse.hip'], cwd='/tmp/dg3', capture_output=True, text=True)
open('/root/repo/tools/diag/solve_phases.patch', 'w').write(r.stdout)
print("patch", len(r.stdout))
