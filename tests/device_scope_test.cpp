// CPU test of the C ABI's device rule (ocean-simulation_amd/csrc/device_scope.h) over a two-device stub
// runtime: the WaterBody lifecycle's entry points -- create, set_params, init, step, read_async,
// readback release, destroy -- each run inside the scope exactly as ocean_abi.cpp wraps them, with the
// caller's thread on device 0 or 1 and the context on device 0 or 1.  Inside every call the context's
// device must be current; after every call the caller's own device must be current again, also when
// the runtime refuses to switch.  Built and run by tests/test_device_scope.py (g++, no HIP).
//   device_scope_test            exit 0 when every check holds, 1 (with the failed check) otherwise
#include <cstdio>
#include <string>

#include "device_scope.h"

namespace {

// Two-device stub of the runtime's per-thread current device.
struct Stub {
    static int current;
    static int devices;
    static int fail_set_to;  // set() to this device fails (-1: never)
    static int sets;         // set() calls
};
int Stub::current = 0, Stub::devices = 2, Stub::fail_set_to = -1, Stub::sets = 0;

struct StubApi {
    static int get(int* d) {
        *d = Stub::current;
        return 0;
    }
    static int set(int d) {
        ++Stub::sets;
        if (d < 0 || d >= Stub::devices) return 101;  // hipErrorInvalidDevice
        if (d == Stub::fail_set_to) return 999;
        Stub::current = d;
        return 0;
    }
};
using Scope = ocean::BasicDeviceScope<StubApi>;

int failures = 0;
void expect(bool ok, const std::string& what) {
    if (!ok) {
        std::printf("FAIL: %s\n", what.c_str());
        ++failures;
    }
}

struct Ctx {
    int device;
};
struct Readback {
    int device;
};

// An entry point as ocean_abi.cpp writes one: the scope first, the work inside it.  `work` checks that
// the context's device is current for the call's whole span; the return value is the call's status.
template <class Work>
int entry(int device, Work&& work) {
    Scope scope(device);
    if (scope.error()) return -4;  // OCEAN_E_DEVICE
    work();
    return 0;
}

void lifecycle(int caller, int dev) {
    const std::string tag = "caller " + std::to_string(caller) + ", context " + std::to_string(dev) + ": ";
    Stub::current = caller;
    auto on_ctx = [&](const char* call) {
        return [=] { expect(Stub::current == dev, tag + call + " ran off the context's device"); };
    };
    auto back = [&](const char* call) { expect(Stub::current == caller, tag + call + " left the caller's device moved"); };
    Ctx ctx{dev};
    expect(entry(dev, on_ctx("ocean_create")) == 0, tag + "ocean_create failed");
    back("ocean_create");
    for (const char* call : {"ocean_set_params", "ocean_generate_noise", "ocean_init_spectrum", "ocean_step",
                             "ocean_read_async", "ocean_readback_wait"}) {
        expect(entry(ctx.device, on_ctx(call)) == 0, tag + call + " failed");
        back(call);
    }
    Readback rb{ctx.device};
    expect(entry(rb.device, on_ctx("ocean_readback_release")) == 0, tag + "ocean_readback_release failed");
    back("ocean_readback_release");
    // a host that moves its own device between calls: every call still restores the caller's current one
    Stub::current = 1 - caller;
    expect(entry(ctx.device, on_ctx("ocean_step")) == 0, tag + "ocean_step failed");
    expect(Stub::current == 1 - caller, tag + "ocean_step after the host switched devices");
    Stub::current = caller;
    expect(entry(ctx.device, on_ctx("ocean_destroy")) == 0, tag + "ocean_destroy failed");
    back("ocean_destroy");
}

}  // namespace

int main() {
    for (int caller = 0; caller < 2; ++caller)
        for (int dev = 0; dev < 2; ++dev) lifecycle(caller, dev);
    // same device: no set at all (ocean.h: hipSetDevice only when the device differs)
    Stub::current = 1;
    Stub::sets = 0;
    { Scope s(1); }
    expect(Stub::sets == 0, "a scope on the current device called set()");
    // the runtime refuses the switch: the error is reported and the caller's device stays, with no restore
    Stub::current = 1;
    Stub::fail_set_to = 0;
    Stub::sets = 0;
    {
        Scope s(0);
        expect(s.error() == 999, "a refused switch did not report the runtime's error");
        expect(Stub::current == 1, "a refused switch moved the device");
    }
    expect(Stub::current == 1 && Stub::sets == 1, "a refused switch was 'restored' (a second set)");
    Stub::fail_set_to = -1;
    // a device the runtime does not have
    {
        Scope s(5);
        expect(s.error() != 0, "an invalid device was accepted");
    }
    expect(Stub::current == 1, "an invalid device moved the caller's device");
    // nested scopes (an entry that calls another entry): each level restores its own caller's device
    Stub::current = 0;
    {
        Scope a(1);
        expect(Stub::current == 1, "outer scope");
        {
            Scope b(0);
            expect(Stub::current == 0, "inner scope");
        }
        expect(Stub::current == 1, "inner scope did not restore the outer call's device");
    }
    expect(Stub::current == 0, "outer scope did not restore the caller's device");
    if (failures) return 1;
    std::printf("ok\n");
    return 0;
}
