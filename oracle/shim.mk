# Builds oracle/_ref/shim_driver: the reference's ingress/egress translation
# units (compiled from /root/reference/src, include order fixed by
# ref_prelude.h, nothing copied) + integration/rk_reference_shim.cpp (the
# binding a maintainer adds) + librepkiller_amd.so.  TEST
# INFRASTRUCTURE: it proves the shim compiles and links against the
# reference's real headers, and the GPU suite runs it end to end.
#
#   make -f oracle/shim.mk            (from the repo root)
REF_SRC ?= /root/reference/src
OUT     := oracle/_ref
CXX     ?= g++
FLAGS   := -std=c++14 -O2 -march=x86-64 -ffp-contract=off \
           -DREF_STRUCTS_H='"$(REF_SRC)/structs.h"' -include oracle/ref_prelude.h \
           -I$(REF_SRC) -Iinclude -Iintegration
LIB_TUS := $(REF_SRC)/FragmentsDatabase.cpp $(REF_SRC)/SequenceOcupationList.cpp \
           $(REF_SRC)/commonFunctions.cpp $(REF_SRC)/class_structs.cpp
SHIM    := integration/rk_reference_shim.cpp integration/shim_driver.cpp

all: $(OUT)/shim_driver

$(OUT):
	mkdir -p $(OUT)

$(OUT)/shim_driver: $(SHIM) integration/rk_reference_shim.h include/repkiller_amd.h \
                    oracle/ref_prelude.h $(LIB_TUS) repkiller_amd/librepkiller_amd.so | $(OUT)
	$(CXX) $(FLAGS) $(SHIM) $(LIB_TUS) -Lrepkiller_amd -lrepkiller_amd \
	    -Wl,-rpath,'$$ORIGIN/../../repkiller_amd' -lpthread -o $@

.PHONY: all
