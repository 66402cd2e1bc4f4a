/* Forced-include prelude for building the reference (estebanpw/repkiller) as a
 * parity/timing oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference's structs.h opens with `#pragma pack(1)` and never closes it
 * (/root/reference/src/structs.h:2), so every class declared after it --
 * including libstdc++'s mutex/condition_variable inside SaverQueue
 * (SaverQueue.h:27-31) -- is laid out packed; on glibc 2.35 the condvar futex
 * then fails and the stock binary aborts before writing output.
 * Pulling every standard header in FIRST, then the reference's structs.h, then
 * restoring the default packing keeps FragFile packed (as the reference wants)
 * while leaving the standard library and SaverQueue with their normal layout.
 * No reference source is copied or replaced: this file only fixes include order.
 */
#include <iostream>
#include <fstream>
#include <cstdlib>
#include <string>
#include <thread>
#include <utility>
#include <queue>
#include <vector>
#include <memory>
#include <algorithm>
#include <sstream>
#include <forward_list>
#include <inttypes.h>
#include <limits>
#include <cmath>
#include <mutex>
#include <condition_variable>
#include <chrono>
#include <stdexcept>
#include REF_STRUCTS_H
#pragma pack()
