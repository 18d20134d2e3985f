// Registry.h — resource registry of one pipeline construction (Registry.h:17-205
// subset used by DDGINode and its consumers): owns buffers/binding sets, publishes
// named resources (unique names, Fatal on duplicates, Registry.h:170-173) and
// carries DDGI history across pipeline rebuilds the way createOrReuseTexture2D
// does (Registry.cpp:120-150): the DDGI context that owns the atlases is adopted
// from the previous registry when its description matches.
#pragma once

#include <memory>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/ark_ddgi.h"
#include "backend/hip/HipBackend.h"

class Registry final {
public:
    Registry(HipBackend&, Registry* previousRegistry);
    ~Registry();
    Registry(const Registry&) = delete;
    Registry& operator=(const Registry&) = delete;

    HipBackend& backend() { return m_backend; }
    void setCurrentNode(std::optional<std::string> node) { m_currentNode = std::move(node); }

    Buffer& createBuffer(const void* data, size_t size, Buffer::Usage);
    template<typename T>
    Buffer& createBufferForData(const T& data, Buffer::Usage usage) { return createBuffer(&data, sizeof(T), usage); }
    Buffer& wrapBuffer(void* devicePtr, size_t size, Buffer::Usage usage);
    Texture& wrapTexture(const std::string& name, void* devicePtr, int width, int height, Texture::Format format);
    BindingSet& createBindingSet(std::vector<ShaderBinding>);

    enum class ReuseMode { Created, Reused };
    // Adopts the previous registry's DDGI context with the same name and description.
    std::pair<ArkDdgiCtx*, ReuseMode> createOrReuseDdgiContext(const std::string& name, const ArkDdgiDesc& desc);

    bool hasPreviousNode(const std::string& name) const;
    void publish(const std::string& name, BindingSet&);
    void publish(const std::string& name, Buffer&);
    BindingSet* getBindingSet(const std::string& name);
    Buffer* getBuffer(const std::string& name);

private:
    struct OwnedCtx {
        std::string name;
        ArkDdgiDesc desc;
        ArkDdgiCtx* ctx;
    };
    HipBackend& m_backend;
    Registry* m_previous;
    std::optional<std::string> m_currentNode;
    std::vector<std::string> m_allNodeNames;
    std::vector<std::unique_ptr<Buffer>> m_buffers;
    std::vector<std::unique_ptr<Texture>> m_textures;
    std::vector<std::unique_ptr<BindingSet>> m_bindingSets;
    std::vector<OwnedCtx> m_ddgiContexts;
    std::unordered_map<std::string, std::pair<BindingSet*, std::string>> m_publishedBindingSets;
    std::unordered_map<std::string, std::pair<Buffer*, std::string>> m_publishedBuffers;
    friend class RenderPipeline;
};
