// Probe (measurement shim, not product): what ds_read_b64_tr_b8 delivers on gfx950, and the
// v_mfma_i32_16x16x64_i8 operand maps, with exact integer data.  Prints, per lane, the LDS byte
// addresses of the 8 bytes each lane receives when lane l supplies address 8*l.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void tr8(int* out, int shift) {
  __shared__ unsigned char lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = (unsigned char)(i >> shift);
  __syncthreads();
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + threadIdx.x * 8));
  out[threadIdx.x * 2] = r[0];
  out[threadIdx.x * 2 + 1] = r[1];
}

// D = A x B with A[i][k] = (k == kk) ? 1 : 0 style probes: A lane l element e = code(l, e); B all ones
// except one element -> read back D to find which (lane, element) pairs multiply.
__global__ void mfma_map(const signed char* a, const signed char* b, int* d) {
  const int l = threadIdx.x;
  v4i av = *reinterpret_cast<const v4i*>(a + 16 * l);
  v4i bv = *reinterpret_cast<const v4i*>(b + 16 * l);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

int main() {
  int* dout;
  hipMalloc(&dout, 64 * 2 * sizeof(int));
  int h[2][128];
  for (int s = 0; s < 2; ++s) {
    tr8<<<1, 64>>>(dout, s ? 8 : 0);
    hipMemcpy(h[s], dout, sizeof(h[s]), hipMemcpyDeviceToHost);
  }
  printf("tr8: lane -> 8 source byte addresses (lane l gave address 8*l)\n");
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 8; ++e) {
      const int lo = (h[0][2 * l + e / 4] >> (8 * (e % 4))) & 255, hi = (h[1][2 * l + e / 4] >> (8 * (e % 4))) & 255;
      printf(" %4d", hi * 256 + lo);
    }
    printf("\n");
  }
  // MFMA map: for each (lane, element) of A set 1 at one position with B = k-code; D[i][j] = sum_k A[i][k] B[k][j]
  signed char ha[1024], hb[1024];
  signed char *da, *db;
  int *dd, hd[256];
  hipMalloc(&da, 1024);
  hipMalloc(&db, 1024);
  hipMalloc(&dd, 1024);
  // probe: A lane la element ea = 1, all else 0; B lane lb element eb = (lb % 16) + 1 for lanes with the
  // same group... simpler: B[lane][e] = e + 16 * (lane >> 4) + 1 (distinct per (group, element)), so the
  // D entries of row (la % 16) reveal which B element met A(la, ea).
  int bad = 0;
  for (int la = 0; la < 64; la += 5)
    for (int ea = 0; ea < 16; ea += 3) {
      for (int i = 0; i < 1024; ++i) ha[i] = 0;
      ha[16 * la + ea] = 1;
      for (int lb = 0; lb < 64; ++lb)
        for (int e = 0; e < 16; ++e) hb[16 * lb + e] = (signed char)(e + 16 * (lb >> 4) + 1 + (lb & 15) * 0);
      hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice);
      hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
      mfma_map<<<1, 64>>>(da, db, dd);
      hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
      // row i = la % 16: D[i][j] for every column j: lane l holds rows 4*(l>>4)+r, col l&15
      const int i = la % 16;
      const int l = (i / 4) * 16 + 0, r = i % 4;
      const int got = hd[4 * l + r];
      const int expect = ea + 16 * (la >> 4) + 1;
      if (got != expect) ++bad;
      printf("A(lane %2d, elem %2d) met B code %3d (same (group, elem) -> %3d)\n", la, ea, got, expect);
    }
  printf("mfma pairing mismatches: %d\n", bad);
  return 0;
}
