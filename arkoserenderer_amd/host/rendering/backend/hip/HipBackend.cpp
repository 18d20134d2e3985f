#include "HipBackend.h"

#include <hip/hip_runtime.h>

#include "core/Logging.h"

Buffer::Buffer(void* devicePtr, size_t size, Usage usage, bool owning)
    : m_ptr(devicePtr), m_size(size), m_usage(usage), m_owning(owning)
{
}

Buffer::~Buffer()
{
    if (m_owning && m_ptr) (void)hipFree(m_ptr);
}

HipBackend::HipBackend(int device)
    : m_device(device)
{
    if (hipSetDevice(device) != hipSuccess) ARKOSE_LOG(Fatal, "HipBackend: hipSetDevice(%d) failed", device);
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) ARKOSE_LOG(Fatal, "HipBackend: stream creation failed");
    m_stream = s;
}

HipBackend::~HipBackend()
{
    if (m_stream) {
        (void)hipStreamSynchronize(static_cast<hipStream_t>(m_stream));
        (void)hipStreamDestroy(static_cast<hipStream_t>(m_stream));
    }
}

void HipBackend::synchronize()
{
    if (hipStreamSynchronize(static_cast<hipStream_t>(m_stream)) != hipSuccess) ARKOSE_LOG(Error, "HipBackend: stream synchronize failed");
}

std::unique_ptr<Buffer> HipBackend::createBuffer(const void* hostData, size_t size, Buffer::Usage usage)
{
    void* p = nullptr;
    if (hipMalloc(&p, size) != hipSuccess) {
        ARKOSE_LOG(Error, "HipBackend: hipMalloc(%zu) failed", size);
        return nullptr;
    }
    if (hostData && hipMemcpy(p, hostData, size, hipMemcpyHostToDevice) != hipSuccess) ARKOSE_LOG(Error, "HipBackend: upload failed");
    return std::make_unique<Buffer>(p, size, usage, true);
}
