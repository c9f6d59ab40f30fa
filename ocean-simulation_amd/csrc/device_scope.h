// The device rule of the C ABI (ocean.h, "Conventions"): every call makes its context's device current
// for its own span and gives the calling thread its own current device back on return, so a host that
// drives several contexts from one thread, or runs torch in the same process, never sees its current
// device move.  The runtime's get / set pair is a template parameter: the library instantiates it with
// hipGetDevice / hipSetDevice (ocean_abi.cpp), and tests/test_device_scope.py with a two-device stub on
// the CPU, so the restore branch is exercised without a second GPU.
//   Api::get(int* device) -> 0 on success;  Api::set(int device) -> 0 on success, else the error code.
#pragma once

namespace ocean {

template <class Api>
class BasicDeviceScope {
  public:
    explicit BasicDeviceScope(int device) {
        if (Api::get(&prev_) != 0) prev_ = -1;
        if (prev_ == device) return;  // already current: nothing to set, nothing to restore
        const int e = Api::set(device);
        if (e != 0) {
            error_ = e;  // the caller's device is still current: nothing to restore
            return;
        }
        restore_ = prev_ >= 0;
    }
    ~BasicDeviceScope() {
        if (restore_) (void)Api::set(prev_);
    }
    BasicDeviceScope(const BasicDeviceScope&) = delete;
    BasicDeviceScope& operator=(const BasicDeviceScope&) = delete;
    // The runtime's error from making the device current (0: it is current).
    int error() const { return error_; }

  private:
    int prev_ = -1;
    bool restore_ = false;
    int error_ = 0;
};

}  // namespace ocean
