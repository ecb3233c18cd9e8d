# Host AddressSanitizer run of the library's host-only C++ (decagon_amd/csrc/layout.cpp:
# dg_staged_order, the bank-conflict-avoiding nonzero order of the staged SpMM) on config P's
# full staged layout — every drug×drug relation, one GPU and the 8-GPU rank-0 share.  CPU only.
#   bash scripts/asan_layout.sh
set -e
cd "$(dirname "$0")/.."
mkdir -p build/asan
g++ -O1 -g -fsanitize=address -fno-omit-frame-pointer -shared -fPIC -Iinclude decagon_amd/csrc/layout.cpp \
  -o build/asan/liblayout_asan.so
LD_PRELOAD=$(g++ -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0 \
  python3 scripts/asan_layout.py build/asan/liblayout_asan.so
