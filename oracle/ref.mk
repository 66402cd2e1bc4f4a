# Builds the reference repkiller from its own sources, where they lie under
# /root/reference/src, into oracle/_ref/.  TEST INFRASTRUCTURE ONLY: the
# outputs are the parity oracle and the CPU baseline; nothing in the product
# links or calls them.  Only the include order is changed (ref_prelude.h);
# no reference source is copied, patched or replaced.
#
#   make -f oracle/ref.mk            (from the repo root)
REF_SRC ?= /root/reference/src
OUT     := oracle/_ref
CXX     ?= g++
# -march=x86-64 matches the shipped binary's DWARF producer (no FMA contraction
# of 0.4*a + 0.6*b, SequenceOcupationList.cpp:30; SURVEY.md §7 "FP exactness").
FLAGS   := -std=c++14 -O3 -march=x86-64 -ffp-contract=off \
           -DREF_STRUCTS_H='"$(REF_SRC)/structs.h"' -include oracle/ref_prelude.h -I$(REF_SRC)
LIB_TUS := $(REF_SRC)/FragmentsDatabase.cpp $(REF_SRC)/SequenceOcupationList.cpp \
           $(REF_SRC)/commonFunctions.cpp $(REF_SRC)/class_structs.cpp

all: $(OUT)/ref_driver $(OUT)/repkiller_fix

$(OUT):
	mkdir -p $(OUT)

# synchronous timing/parity driver (oracle/ref_driver.cpp + the four library TUs)
$(OUT)/ref_driver: oracle/ref_driver.cpp oracle/ref_prelude.h $(LIB_TUS) | $(OUT)
	$(CXX) $(FLAGS) oracle/ref_driver.cpp $(LIB_TUS) -lpthread -o $@

# the reference's own main() (repkiller.cpp) + SaverQueue, layout-fixed
$(OUT)/repkiller_fix: oracle/ref_prelude.h $(LIB_TUS) | $(OUT)
	$(CXX) $(FLAGS) $(REF_SRC)/SaverQueue.cpp $(LIB_TUS) $(REF_SRC)/repkiller.cpp -lpthread -o $@

.PHONY: all
