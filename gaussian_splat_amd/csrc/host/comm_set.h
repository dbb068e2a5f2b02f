// comm_set.h — release of a group's RCCL communicators (group.cpp).
//
// Every handle is released exactly once: by abort after a collective failure
// (comm_failure) or by destroy when the group goes away, never both.  A
// released slot is cleared, so a later teardown skips it.  Header-only and
// templated on the handle type so the rule is unit-tested on the CPU with
// stub handles (tests/host/comm_set_test.cpp, tests/test_host.py).
#pragma once

#include <vector>

namespace gscomm {

template <typename C, typename F>
void abort_all(std::vector<C>& comms, F&& abort_fn) {
    for (C& c : comms)
        if (c) {
            (void)abort_fn(c);
            c = nullptr;
        }
}

template <typename C, typename F>
void destroy_all(std::vector<C>& comms, F&& destroy_fn) {
    for (C& c : comms)
        if (c) {
            (void)destroy_fn(c);
            c = nullptr;
        }
    comms.clear();
}

}  // namespace gscomm
