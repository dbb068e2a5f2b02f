// CPU test of the communicator release rule (gaussian_splat_amd/csrc/host/
// comm_set.h, used by group.cpp): after a collective failure aborts every
// communicator, the group's teardown must not release any of them again
// (a second ncclCommAbort on the freed handles).  Stub handles
// count how often each is aborted or destroyed.  Exit status 0 = pass.
#include <cstdio>
#include <vector>

#include "comm_set.h"

struct Stub {
    int aborts = 0, destroys = 0;
};

static int check(const std::vector<Stub>& s, int aborts, int destroys, const char* what) {
    for (size_t i = 0; i < s.size(); ++i)
        if (s[i].aborts != aborts || s[i].destroys != destroys) {
            std::printf("FAIL %s: handle %zu aborted %d destroyed %d (want %d / %d)\n", what, i, s[i].aborts,
                        s[i].destroys, aborts, destroys);
            return 1;
        }
    return 0;
}

int main() {
    auto ab = [](Stub* c) { return ++c->aborts; };
    auto de = [](Stub* c) { return ++c->destroys; };
    int bad = 0;
    {  // failure, a repeated failure report, then teardown
        std::vector<Stub> s(4);
        std::vector<Stub*> comms;
        for (auto& x : s) comms.push_back(&x);
        gscomm::abort_all(comms, ab);
        gscomm::abort_all(comms, ab);  // (a second failing wait)
        gscomm::destroy_all(comms, de);
        bad |= check(s, 1, 0, "abort then teardown");
        bad |= comms.empty() ? 0 : 1;
    }
    {  // clean teardown
        std::vector<Stub> s(3);
        std::vector<Stub*> comms;
        for (auto& x : s) comms.push_back(&x);
        gscomm::destroy_all(comms, de);
        gscomm::destroy_all(comms, de);
        bad |= check(s, 0, 1, "teardown");
    }
    {  // a partially created set (init failed half way): null slots skipped
        std::vector<Stub> s(2);
        std::vector<Stub*> comms = {&s[0], nullptr, &s[1], nullptr};
        gscomm::abort_all(comms, ab);
        gscomm::destroy_all(comms, de);
        bad |= check(s, 1, 0, "partial set");
    }
    std::printf(bad ? "comm_set: FAIL\n" : "comm_set: ok\n");
    return bad;
}
