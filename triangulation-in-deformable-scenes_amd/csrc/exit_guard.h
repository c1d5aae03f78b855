// exit_guard.h — device contexts a caller never destroyed are released at process exit, while the
// HIP runtime is still alive.
//
// A context holds streams, events, pinned host buffers, device allocations and possibly an RCCL
// communicator.  If the process exits with one still live (a Python interpreter tearing down without
// running __del__, a C++ caller that never calls deftri_ctx_destroy), those resources would otherwise
// meet the runtime's own static teardown — and a profiler's tool library finalizing in its own exit
// handler — in an order nobody controls.  The first device context registers one std::atexit
// handler; the runtime initialized before that (hipGetDeviceCount / hipSetDevice ran first), so its
// static destructors were registered earlier and run later than the handler: the handler destroys
// the still-live contexts first.  Creation and destruction keep the set; the handler empties it.
#pragma once

#include <cstdlib>
#include <mutex>
#include <unordered_set>

namespace deftri {

template <class Ctx, int (*Destroy)(Ctx *)>
class LiveContexts {
public:
    static void add(Ctx *c) {
        std::lock_guard<std::mutex> g(mu());
        set().insert(c);
        static const bool registered = (std::atexit(&LiveContexts::release_all), true);
        (void)registered;
    }
    static void remove(Ctx *c) {
        std::lock_guard<std::mutex> g(mu());
        set().erase(c);
    }

private:
    static std::mutex &mu() {
        static std::mutex *m = new std::mutex;          // never destroyed: usable from the exit handler
        return *m;
    }
    static std::unordered_set<Ctx *> &set() {
        static auto *s = new std::unordered_set<Ctx *>;
        return *s;
    }
    static void release_all() {
        std::unordered_set<Ctx *> live;
        {
            std::lock_guard<std::mutex> g(mu());
            live.swap(set());
        }
        for (Ctx *c : live) Destroy(c);                 // Destroy's own remove() finds nothing left
    }
};

}  // namespace deftri
