# build_variant.sh NAME "EXTRA HIPCC FLAGS" [KERNEL_SOURCE]: variants/NAME/liblda_mi355x.so (A/B runs via LDA_MI355X_LIB)
set -e
cd "$(dirname "$0")/.."
D=variants/$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2 -I ldagibbssampling_amd/csrc -c ${3:-ldagibbssampling_amd/csrc/lda_kernels.hip} -o $D/k.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2 -I ldagibbssampling_amd/csrc -x hip -c ldagibbssampling_amd/csrc/lda_capi.cpp -o $D/c.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/liblda_mi355x.so $D/k.o $D/c.o ldagibbssampling_amd/csrc/build/lda_dirichlet.o
rm -f $D/k.o $D/c.o
