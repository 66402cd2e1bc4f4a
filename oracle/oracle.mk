# Builds the CPU restatement (TEST INFRASTRUCTURE ONLY) into oracle/_build/.
#   make -f oracle/oracle.mk     (from the repo root)
OUT    := oracle/_build
CC     ?= gcc
CFLAGS := -std=gnu11 -O2 -march=x86-64 -ffp-contract=off -fno-fast-math -Wall -Wextra -fPIC

all: $(OUT)/librk_oracle.so $(OUT)/rk_oracle

$(OUT):
	mkdir -p $(OUT)

$(OUT)/librk_oracle.so: oracle/rk_oracle.c oracle/rk_oracle.h | $(OUT)
	$(CC) $(CFLAGS) -shared oracle/rk_oracle.c -lm -o $@

$(OUT)/rk_oracle: oracle/rk_oracle_main.c oracle/rk_oracle.c oracle/rk_oracle.h | $(OUT)
	$(CC) $(CFLAGS) oracle/rk_oracle_main.c oracle/rk_oracle.c -lm -o $@

.PHONY: all
