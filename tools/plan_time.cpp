// Host plan build time of the 9-mer lattice (tool): kp::build_plan three times.
#include <chrono>
#include <cstdio>
#include "kp_plan.h"
int main(){ kp::host_plan P; for(int r=0;r<3;++r){auto t0=std::chrono::steady_clock::now();
 std::string e=kp::build_plan("NNNNMNNNN", 4096, P);
 double ms=std::chrono::duration<double,std::milli>(std::chrono::steady_clock::now()-t0).count();
 printf("%s %.2f ms nblocks=%llu B=%u\n", e.c_str(), ms, (unsigned long long)P.g.nblocks, P.g.B);} }
