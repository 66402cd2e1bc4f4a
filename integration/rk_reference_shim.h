// rk_reference_shim.h -- the binding a repkiller maintainer adds to the
// reference to run its hot path on an MI355X through librepkiller_amd.so.
//
// classify_on_gpu() replaces lines 83-92 of execWithParams
// (/root/reference/src/repkiller.cpp:80-97): generate_fragment_groups
// (commonFunctions.h:35), generate_diagonal_func (:59) and sort_groups (:57).
// It takes the reference's own FragmentsDatabase / sequence_manager
// (FragmentsDatabase.h:14-34, structs.h:79-91) and returns the FGList its
// SaverQueue (SaverQueue.h:37-41) writes -- groups in creation order, members
// in sorted order -- so ingress and egress stay the reference's code.
//
// Build: compiled against the reference's headers (with the include-order
// prelude oracle/ref_prelude.h, see there) and linked with
// -L<repo>/repkiller_amd -lrepkiller_amd; oracle/shim.mk does exactly that.
#pragma once
#include "FragmentsDatabase.h"

// throws runtime_error on any rk_status (the reference's exception type)
FGList *classify_on_gpu(const FragmentsDatabase &frag_db, const sequence_manager &sm,
                        double len_ratio, double pos_ratio);
