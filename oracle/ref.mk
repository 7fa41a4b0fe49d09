# oracle/ref.mk — compile the reference's OWN sources (in place, read-only)
# into oracle/_ref/ so the CPU restatement can be pinned against them.
#   libblst_ref.so   : lib/blst/src/server.c + assembly.S, flags as
#                      plonk-core/build.rs:38-54 (-mno-avx -fno-builtin)
#   libstrobe_ref.so : lib/PLONK/src/transcript/strobe.cpp + our Merlin
#                      framing shim (ref_strobe_shim.cpp)
# Nothing under /root/reference is copied; outputs go only to oracle/_ref/.
REF     ?= /root/reference/Prize 1B/plonk-core/lib
OUT     := _ref
BLST    := $(REF)/blst
STROBE  := $(REF)/PLONK/src/transcript

all: $(OUT)/libblst_ref.so $(OUT)/libstrobe_ref.so

$(OUT):
	mkdir -p $(OUT)

$(OUT)/libblst_ref.so: | $(OUT)
	gcc -O2 -fPIC -mno-avx -fno-builtin -Wno-unused-function \
	    -I"$(BLST)/include" -c "$(BLST)/src/server.c" -o $(OUT)/server.o
	gcc -O2 -fPIC -mno-avx -c "$(BLST)/src/assembly.S" -o $(OUT)/assembly.o
	gcc -shared -o $@ $(OUT)/server.o $(OUT)/assembly.o

$(OUT)/libstrobe_ref.so: ref_strobe_shim.cpp | $(OUT)
	g++ -O2 -fPIC -std=c++17 -I"$(STROBE)" -shared -o $@ \
	    "$(STROBE)/strobe.cpp" ref_strobe_shim.cpp

.PHONY: all
