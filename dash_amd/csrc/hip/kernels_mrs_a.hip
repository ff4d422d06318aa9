// Mixed-radix chain kernels for CRT sizes 7 (templates: mrs_chain.h). One unit per few K keeps
// every unit's build short and lets them compile in parallel.
#include "mrs_chain.h"

namespace dash {
namespace dev {

template void launch_mrs_chain_k<7>(const MrsArgs&, const Act&, int, const ModC*, const AesGlobals&, hipStream_t);

}  // namespace dev
}  // namespace dash
