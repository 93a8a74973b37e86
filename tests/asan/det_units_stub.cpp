// The ASan ABI check links core.hip, tome.hip and prune.hip only; core.hip's
// mmt_set_deterministic also calls the deterministic-mode setters of the units not linked here
// (attention, glue, norm, stem). They are never reached by abi_host_driver.cpp; these stand-ins
// only satisfy the linker (test infrastructure, not part of libmmt_hip).
namespace mmt {
struct DetState;
int det_set_attention(const DetState&) { return 0; }
int det_set_glue(const DetState&) { return 0; }
int det_set_norm(const DetState&) { return 0; }
int det_set_stem(const DetState&) { return 0; }
}  // namespace mmt
