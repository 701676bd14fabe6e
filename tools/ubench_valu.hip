// tools/ubench_valu.hip -- measure gfx950 VALU issue rates of the integer
// instructions the verify kernels are built from (the roofline denominator,
// BASELINE.md "Roofline framing": v_mad_i64_i32 issue rate x 256 CU x clock).
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu && tools/ubench_valu [lone]
//
// Each kernel runs 16 independent dependency chains per lane of one
// instruction (inline asm, so nothing is folded), 8 waves per SIMD.
// Prints lane-ops per second and per CU-clock (clock from the kernel's own
// s_memtime / s_memrealtime ratio).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 16

template<int OP>
__global__ void __launch_bounds__(256) k_rate( uint64_t * out, int iters, uint64_t * clk ) {
  uint64_t acc[CH];
  uint32_t a = threadIdx.x * 2654435761u + blockIdx.x, b = a ^ 0x9e3779b9u;
#pragma unroll
  for( int k=0; k<CH; k++ ) acc[k] = ((uint64_t)(a + k) << 32) | (b + 3*k);
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for( int i=0; i<iters; i++ ) {
#pragma unroll
    for( int k=0; k<CH; k++ ) {
      if( OP==0 ) { uint64_t sd; asm volatile( "v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sd) : "v"(a), "v"(b) ); }
      if( OP==1 ) { uint64_t sd; asm volatile( "v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sd) : "v"(a), "v"(b) ); }
      if( OP==2 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
      if( OP==3 ) { asm volatile( "v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k+1)%CH]) ); }
      if( OP==4 ) { asm volatile( "v_ashrrev_i64 %0, 3, %0" : "+v"(acc[k]) ); }
      if( OP==5 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
      if( OP==6 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_mul_u32_u24 %0, %0, %1" : "+v"(lo) : "v"(b) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
      if( OP==7 ) { double d = __longlong_as_double( acc[k] ); asm volatile( "v_fma_f64 %0, %0, %1, %0" : "+v"(d) : "v"(__longlong_as_double( (uint64_t)b )) ); acc[k] = __double_as_longlong( d ); }
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t x = 0;
#pragma unroll
  for( int k=0; k<CH; k++ ) x ^= acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if( threadIdx.x == 0 && blockIdx.x == 0 ) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template<int OP>
static void run( char const * name ) {
  int nb = 256 * 8;   // 8 blocks of 256 per CU = 32 waves / CU
  int iters = 2000;
  uint64_t *out, *clk;
  (void)hipMalloc( &out, 8UL * nb * 256 ); (void)hipMalloc( &clk, 16 );
  hipLaunchKernelGGL( k_rate<OP>, dim3(nb), dim3(256), 0, 0, out, 10, clk );
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate( &e0 ); (void)hipEventCreate( &e1 );
  (void)hipEventRecord( e0 );
  hipLaunchKernelGGL( k_rate<OP>, dim3(nb), dim3(256), 0, 0, out, iters, clk );
  (void)hipEventRecord( e1 ); (void)hipEventSynchronize( e1 );
  float ms; (void)hipEventElapsedTime( &ms, e0, e1 );
  uint64_t c[2]; (void)hipMemcpy( c, clk, 16, hipMemcpyDeviceToHost );
  double ops = (double)nb * 256 * iters * CH;
  double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;   // s_memrealtime ticks at 100 MHz
  double per_cu_clk = ops / (ms * 1e-3) / 256.0 / (ghz * 1e9);
  printf( "%-16s %8.3f ms  %10.3f Tops/s  clock %.2f GHz  %6.1f lane-ops/clk/CU\n", name, ms, ops / (ms * 1e-3) / 1e12, ghz, per_cu_clk );
  (void)hipFree( out ); (void)hipFree( clk );
}

/* One wave alone on the chip (one 64-lane block): cycles per instruction
   (s_memtime) with NC independent chains per lane -- NC = 1 is the
   dependent latency, large NC the lone wave's issue interval (the regime of
   the latency kernels, one wave per SIMD). */
template<int OP, int NC>
__global__ void __launch_bounds__(64) k_lone( uint64_t * out, int iters, uint64_t * clk ) {
  uint64_t acc[NC];
  uint32_t a = threadIdx.x * 2654435761u, b = a ^ 0x9e3779b9u;
#pragma unroll
  for( int k=0; k<NC; k++ ) acc[k] = ((uint64_t)(a + k) << 32) | (b + 3*k);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for( int i=0; i<iters; i++ ) {
#pragma unroll
    for( int k=0; k<NC; k++ ) {
      if( OP==0 ) { uint64_t sd; asm volatile( "v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sd) : "v"(a), "v"(b) ); }
      if( OP==3 ) { asm volatile( "v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k+1)%NC]) ); }
      if( OP==4 ) { asm volatile( "v_ashrrev_i64 %0, 3, %0" : "+v"(acc[k]) ); }
      if( OP==5 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
      if( OP==8 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_cndmask_b32 %0, %0, %1, vcc" : "+v"(lo) : "v"(b) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
      if( OP==9 ) { uint32_t lo = (uint32_t)acc[k]; asm volatile( "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(lo) ); acc[k] = (acc[k] & ~0xffffffffull) | lo; }
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t x = 0;
#pragma unroll
  for( int k=0; k<NC; k++ ) x ^= acc[k];
  out[threadIdx.x] = x;
  if( threadIdx.x == 0 ) clk[0] = t1 - t0;
}

template<int OP, int NC>
static void lone( char const * name ) {
  uint64_t *out, *clk;
  int iters = 4000;
  (void)hipMalloc( &out, 8UL * 64 ); (void)hipMalloc( &clk, 16 );
  hipLaunchKernelGGL( (k_lone<OP, NC>), dim3(1), dim3(64), 0, 0, out, 10, clk );
  hipLaunchKernelGGL( (k_lone<OP, NC>), dim3(1), dim3(64), 0, 0, out, iters, clk );
  (void)hipDeviceSynchronize();
  uint64_t c; (void)hipMemcpy( &c, clk, 8, hipMemcpyDeviceToHost );
  printf( "lone wave %-16s %2d chains  %6.2f cycles per instruction\n", name, NC, (double)c / ((double)iters * NC) );
  (void)hipFree( out ); (void)hipFree( clk );
}

int main( int argc, char ** argv ) {
  if( argc > 1 ) {   /* "lone": the one-wave table */
    lone<0,1>( "v_mad_i64_i32" ); lone<0,2>( "v_mad_i64_i32" ); lone<0,5>( "v_mad_i64_i32" ); lone<0,16>( "v_mad_i64_i32" );
    lone<3,1>( "v_lshl_add_u64" ); lone<3,16>( "v_lshl_add_u64" );
    lone<4,1>( "v_ashrrev_i64" ); lone<4,16>( "v_ashrrev_i64" );
    lone<5,1>( "v_add_u32" ); lone<5,16>( "v_add_u32" );
    lone<8,1>( "v_cndmask_b32" ); lone<8,16>( "v_cndmask_b32" );
    lone<9,1>( "v_mov_b32_dpp" ); lone<9,16>( "v_mov_b32_dpp" );
    return 0;
  }
  run<0>( "v_mad_i64_i32" );
  run<1>( "v_mad_u64_u32" );
  run<2>( "v_mul_lo_u32" );
  run<3>( "v_lshl_add_u64" );
  run<4>( "v_ashrrev_i64" );
  run<5>( "v_add_u32" );
  run<6>( "v_mul_u32_u24" );
  run<7>( "v_fma_f64" );
  return 0;
}
