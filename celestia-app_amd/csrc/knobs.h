// Environment knobs of libcda.
//
// The product library (libcda.so) reads only the deployer knobs -- the ones a
// node operator may need:
//   CDA_SYNC_CHECK       synchronise after every stage (fault attribution)
//   CDA_HOST_THREADS     host threads of the host-buffer entry points
//   CDA_HOST_REGISTER    pin (hipHostRegister) caller buffers of host batches
//   CDA_HOST_PIPE_CHUNK  squares per chunk of the host-buffer pipeline (host RAM)
//   CDA_PIPELINE_CHUNK   squares per RS chunk of a device batch
// Every schedule threshold and A/B switch is a constant in the product build.
// The test build (libcda_test.so: `make test-lib`, -DCDA_TESTING) additionally
// reads the test knobs -- fault injection (CDA_FAULT, CDA_COMM_FAULT) and the
// A/B schedule switches the parity tests use to reach every alternative
// schedule -- so a variable left in a node's environment cannot change what
// libcda.so computes or make it fail.
#pragma once
#include <cstdlib>

namespace cda {

inline const char* deploy_knob(const char* name) { return std::getenv(name); }

#ifdef CDA_TESTING
inline constexpr bool kTestBuild = true;
inline const char* test_knob(const char* name) { return std::getenv(name); }
#else
inline constexpr bool kTestBuild = false;
inline const char* test_knob(const char*) { return nullptr; }
#endif

}  // namespace cda
