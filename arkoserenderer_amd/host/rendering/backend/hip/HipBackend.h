// HipBackend.h — the minimal rendering/backend/hip compute backend the DDGI node
// needs: one GPU, one HIP stream per frame's command list, device buffers and
// textures as plain device views. It replaces the Vulkan backend's role for this
// path (Backend.h:20-113 / CommandList.h:9-104 subset); no raster, no RT pipeline.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

struct HipStreamHandle; // opaque (hipStream_t)

class Buffer {
public:
    enum class Usage { ConstantBuffer, StorageBuffer };
    Buffer(void* devicePtr, size_t size, Usage usage, bool owning);
    ~Buffer();
    Buffer(const Buffer&) = delete;
    Buffer& operator=(const Buffer&) = delete;
    void* devicePointer() const { return m_ptr; }
    size_t size() const { return m_size; }
    Usage usage() const { return m_usage; }
    void setName(std::string n) { m_name = std::move(n); }
    const std::string& name() const { return m_name; }
    void setStride(size_t s) { m_stride = s; }
    size_t stride() const { return m_stride; }

private:
    void* m_ptr;
    size_t m_size;
    Usage m_usage;
    bool m_owning;
    size_t m_stride { 0 };
    std::string m_name;
};

class Texture {
public:
    enum class Format { RGBA16F, RG16F };
    Texture(void* devicePtr, int width, int height, Format format) : m_ptr(devicePtr), m_width(width), m_height(height), m_format(format) {}
    void* devicePointer() const { return m_ptr; }
    int width() const { return m_width; }
    int height() const { return m_height; }
    Format format() const { return m_format; }
    void setName(std::string n) { m_name = std::move(n); }
    const std::string& name() const { return m_name; }

private:
    void* m_ptr;
    int m_width, m_height;
    Format m_format;
    std::string m_name;
};

struct ShaderBinding {
    enum class Type { ConstantBuffer, StorageBuffer, SampledTexture };
    Type type;
    Buffer* buffer { nullptr };
    Texture* texture { nullptr };
    static ShaderBinding constantBuffer(Buffer& b) { return { Type::ConstantBuffer, &b, nullptr }; }
    static ShaderBinding storageBuffer(Buffer& b) { return { Type::StorageBuffer, &b, nullptr }; }
    static ShaderBinding sampledTexture(Texture& t) { return { Type::SampledTexture, nullptr, &t }; }
};

class BindingSet {
public:
    explicit BindingSet(std::vector<ShaderBinding> b) : m_bindings(std::move(b)) {}
    const std::vector<ShaderBinding>& bindings() const { return m_bindings; }
    void setName(std::string n) { m_name = std::move(n); }

private:
    std::vector<ShaderBinding> m_bindings;
    std::string m_name;
};

// Command list = the frame's HIP stream; nodes enqueue device work on it.
class CommandList {
public:
    explicit CommandList(void* hipStream) : m_stream(hipStream) {}
    void* hipStream() const { return m_stream; }

private:
    void* m_stream;
};

// Upload staging (kept for the ExecuteCallback signature; DDGI uploads nothing per frame).
class UploadBuffer {
};

class HipBackend {
public:
    explicit HipBackend(int device);
    ~HipBackend();
    HipBackend(const HipBackend&) = delete;
    HipBackend& operator=(const HipBackend&) = delete;
    int device() const { return m_device; }
    void* stream() const { return m_stream; }
    void synchronize();
    std::unique_ptr<Buffer> createBuffer(const void* hostData, size_t size, Buffer::Usage usage);

private:
    int m_device;
    void* m_stream { nullptr };
};
