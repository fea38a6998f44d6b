// dofs_knobs.h — the product library's runtime knobs: the DOFS_* environment variables it reads, all of
// them, validated when a context is created (dofs_create). An unknown DOFS_* name or an invalid value makes
// dofs_create fail (NULL; dofs_last_error(NULL) says which), so a misspelt or retired knob can never select
// a path silently. Each knob and the GPU test that runs it: DESIGN.md §5 "Runtime knobs".
#pragma once

#include <stdlib.h>
#include <string.h>

#include <string>

extern char** environ;

namespace dofs {

struct Knobs {
    int serial = 0;      // DOFS_SERIAL=1: a batch's two stages back to back on one stream (clean per-kernel profiles)
    int flow_long = 0;   // DOFS_FLOW_LONG: long-path replay workers (waves, 4 .. 1024; 0 = the backend's default, 256)
    int long_path = 0;   // DOFS_LONG_PATH: merges from which a heavy path is replayed by a whole wave (16 .. 65536)
    int krt_dnc = -1;    // DOFS_KRT_DNC: 0 the per-frame sweep KRT, 1 the top-down global depths (-1 auto)
    int pre_jump = 8;    // DOFS_PRE_JUMP: batches of at most this many frames take the chip-wide preorder
    int skip_b = 0;      // DOFS_SKIP_B (measurement builds only, -DDOFS_MEASURE): the graph stage alone
    int skip_mask = 0;   // DOFS_SKIPMASK (measurement builds only): 1 short replay, 2 long replay, 4 lift
#ifdef DOFS_MEASURE
    int b_delay_us = 0;  // DOFS_B_DELAY (measurement builds only): stage B of each batch starts this much later
#endif
};

// integer value of v in [lo, hi] (the whole string), else false
inline bool knob_int(const char* v, int lo, int hi, int* out) {
    if (!v || !*v) return false;
    char* end = nullptr;
    const long x = strtol(v, &end, 10);
    if (*end || x < lo || x > hi) return false;
    *out = (int)x;
    return true;
}

// Read every DOFS_* variable of the environment into *out (the new context's own copy: no process-global
// state, so concurrent dofs_create calls and contexts created under different environments keep their own
// knobs); false (and *err) on an unknown name or an invalid value. DOFS_LIB (the Python loader's library
// path) is not the library's and is passed over.
inline bool knobs_load(Knobs* out, std::string* err) {
    Knobs k;
    for (char** e = environ; e && *e; ++e) {
        const char* s = *e;
        if (strncmp(s, "DOFS_", 5) != 0) continue;
        const char* eq = strchr(s, '=');
        if (!eq) continue;
        const std::string name(s, (size_t)(eq - s));
        const char* v = eq + 1;
        bool ok = true;
        if (name == "DOFS_LIB") continue;
        if (name == "DOFS_SERIAL")
            ok = knob_int(v, 0, 1, &k.serial);
        else if (name == "DOFS_FLOW_LONG")
            ok = knob_int(v, 4, 1024, &k.flow_long);
        else if (name == "DOFS_LONG_PATH")
            ok = knob_int(v, 16, 65536, &k.long_path);
        else if (name == "DOFS_KRT_DNC")
            ok = knob_int(v, 0, 1, &k.krt_dnc);
        else if (name == "DOFS_PRE_JUMP")
            ok = knob_int(v, 0, 1 << 20, &k.pre_jump);
#ifdef DOFS_MEASURE
        else if (name == "DOFS_SKIP_B")
            ok = knob_int(v, 0, 1, &k.skip_b);
        else if (name == "DOFS_SKIPMASK")
            ok = knob_int(v, 0, 7, &k.skip_mask);
        else if (name == "DOFS_B_DELAY")
            ok = knob_int(v, 0, 200000, &k.b_delay_us);
#endif
        else {
            if (err) *err = name + " is not a knob of this library (DESIGN.md §5 lists them)";
            return false;
        }
        if (!ok) {
            if (err) *err = name + "=" + v + " is not a valid value";
            return false;
        }
    }
    *out = k;
    return true;
}

}  // namespace dofs
