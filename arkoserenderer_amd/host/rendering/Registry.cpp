#include "Registry.h"

#include <cstring>

#include "core/Logging.h"

Registry::Registry(HipBackend& backend, Registry* previousRegistry)
    : m_backend(backend), m_previous(previousRegistry)
{
}

Registry::~Registry()
{
    for (OwnedCtx& c : m_ddgiContexts)
        if (c.ctx) ark_ddgi_destroy(c.ctx);
}

Buffer& Registry::createBuffer(const void* data, size_t size, Buffer::Usage usage)
{
    m_buffers.push_back(m_backend.createBuffer(data, size, usage));
    if (!m_buffers.back()) ARKOSE_LOG(Fatal, "Registry: buffer creation failed");
    return *m_buffers.back();
}

Buffer& Registry::wrapBuffer(void* devicePtr, size_t size, Buffer::Usage usage)
{
    m_buffers.push_back(std::make_unique<Buffer>(devicePtr, size, usage, false));
    return *m_buffers.back();
}

Texture& Registry::wrapTexture(const std::string& name, void* devicePtr, int width, int height, Texture::Format format)
{
    m_textures.push_back(std::make_unique<Texture>(devicePtr, width, height, format));
    m_textures.back()->setName(name);
    return *m_textures.back();
}

BindingSet& Registry::createBindingSet(std::vector<ShaderBinding> bindings)
{
    m_bindingSets.push_back(std::make_unique<BindingSet>(std::move(bindings)));
    return *m_bindingSets.back();
}

std::pair<ArkDdgiCtx*, Registry::ReuseMode> Registry::createOrReuseDdgiContext(const std::string& name, const ArkDdgiDesc& desc)
{
    if (m_previous) {
        for (OwnedCtx& old : m_previous->m_ddgiContexts) {
            if (old.ctx && old.name == name) {
                if (std::memcmp(&old.desc, &desc, sizeof(desc)) != 0) break; // different grid: recreate (history lost, like a new texture)
                m_ddgiContexts.push_back(old);
                old.ctx = nullptr; // adopted
                return { m_ddgiContexts.back().ctx, ReuseMode::Reused };
            }
        }
    }
    ArkDdgiCtx* ctx = nullptr;
    int rc = ark_ddgi_create(&desc, &ctx);
    if (rc != ARK_DDGI_OK) {
        ARKOSE_LOG(Error, "Registry: ark_ddgi_create failed (%d)", rc);
        return { nullptr, ReuseMode::Created };
    }
    m_ddgiContexts.push_back({ name, desc, ctx });
    return { ctx, ReuseMode::Created };
}

bool Registry::hasPreviousNode(const std::string& name) const
{
    for (const std::string& n : m_allNodeNames)
        if (n == name) return true;
    return false;
}

void Registry::publish(const std::string& name, BindingSet& set)
{
    ARKOSE_ASSERT(m_currentNode.has_value());
    if (m_publishedBindingSets.count(name))
        ARKOSE_LOG(Fatal, "Registry: resource '%s' published twice (node '%s')", name.c_str(), m_currentNode->c_str());
    m_publishedBindingSets[name] = { &set, *m_currentNode };
    set.setName(name);
}

void Registry::publish(const std::string& name, Buffer& buffer)
{
    ARKOSE_ASSERT(m_currentNode.has_value());
    if (m_publishedBuffers.count(name))
        ARKOSE_LOG(Fatal, "Registry: resource '%s' published twice (node '%s')", name.c_str(), m_currentNode->c_str());
    m_publishedBuffers[name] = { &buffer, *m_currentNode };
    buffer.setName(name);
}

BindingSet* Registry::getBindingSet(const std::string& name)
{
    auto it = m_publishedBindingSets.find(name);
    return it == m_publishedBindingSets.end() ? nullptr : it->second.first;
}

Buffer* Registry::getBuffer(const std::string& name)
{
    auto it = m_publishedBuffers.find(name);
    return it == m_publishedBuffers.end() ? nullptr : it->second.first;
}
